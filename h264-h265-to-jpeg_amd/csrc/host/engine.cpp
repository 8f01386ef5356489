// Batch engine: host entropy threads -> HBM job records -> HIP pixel
// pipeline -> host Huffman.  One engine per process per GPU; the IDecoder
// facade and the C ABI (include/h2j.h) both run on it.
//
// Per batch:
//   1. parse      — pool threads run the H.264/H.265 entropy decoders
//                   (hevc_parser.cpp / h264_parser.cpp) into FrameJobs
//   2. pack + H2D — job records packed into one pinned staging buffer, one copy
//   3. GPU        — K1 recon, K2 deblock, K3 SAO, K4 JPEG (h2j_kernels.hip)
//   4. D2H        — quantised coefficients + per-frame statistics
//   5. huffman    — pool threads assemble the JPEG files (jpeg_writer.cpp)
// This is what the reference does per call inside FFmpeg between
// avcodec_send_packet (/root/reference/src/Decoder.cpp:324) and
// av_write_frame (/root/reference/src/Encoder.cpp:278).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "bitstream.h"
#include "h2j.h"
#include "h2j_gpu.h"
#include "job.h"
#include "jpeg_writer.h"

namespace h2j {
namespace {

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

class ThreadPool {
public:
    explicit ThreadPool(int n) : stop_(false), gen_(0), pending_(0) {
        for (int i = 0; i < n; i++) workers_.emplace_back([this] { loop(); });
    }
    ~ThreadPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }
    int size() const { return static_cast<int>(workers_.size()); }
    // run f(i) for i in [0, n) on the pool (caller participates)
    void parallel_for(int n, const std::function<void(int)>& f) {
        if (n <= 0) return;
        if (workers_.empty() || n == 1) {
            for (int i = 0; i < n; i++) f(i);
            return;
        }
        std::atomic<int> next(0);
        auto body = [&]() {
            for (;;) {
                int i = next.fetch_add(1);
                if (i >= n) break;
                f(i);
            }
        };
        {
            std::lock_guard<std::mutex> g(m_);
            task_ = body;
            pending_ = static_cast<int>(workers_.size());
            gen_++;
        }
        cv_.notify_all();
        body();
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this] { return pending_ == 0; });
        task_ = nullptr;
    }

private:
    void loop() {
        unsigned long seen = 0;
        for (;;) {
            std::function<void()> t;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                t = task_;
            }
            if (t) t();
            {
                std::lock_guard<std::mutex> g(m_);
                if (--pending_ == 0) done_.notify_all();
            }
        }
    }
    std::vector<std::thread> workers_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    std::function<void()> task_;
    bool stop_;
    unsigned long gen_;
    int pending_;
};

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool ensure(size_t n) {
        if (n <= cap) return true;
        if (p) h2j_gpu_free(p);
        cap = std::max(n, cap + cap / 2);
        p = h2j_gpu_malloc(cap);
        if (!p) cap = 0;
        return p != nullptr;
    }
    void release() {
        if (p) h2j_gpu_free(p);
        p = nullptr;
        cap = 0;
    }
};

struct HostBuf {
    uint8_t* p = nullptr;
    size_t cap = 0;
    bool ensure(size_t n) {
        if (n <= cap) return true;
        if (p) h2j_gpu_host_free(p);
        cap = std::max(n, cap + cap / 2);
        p = static_cast<uint8_t*>(h2j_gpu_host_alloc(cap));
        if (!p) cap = 0;
        return p != nullptr;
    }
    void release() {
        if (p) h2j_gpu_host_free(p);
        p = nullptr;
        cap = 0;
    }
};

int parse_any(const uint8_t* d, size_t n, FrameJob& job) {
    const int codec = detect_codec(d, n);
    if (codec == 265) return hevc_parse_picture(d, n, job);
    if (codec == 264) return h264_parse_picture(d, n, job);
    job.clear();
    job.error = -100;
    job.message = "not an H.264/H.265 Annex-B stream";
    return -100;
}

}  // namespace

struct Engine {
    int device = 0;
    void* stream = nullptr;
    ThreadPool* pool = nullptr;
    std::string err;
    std::vector<FrameJob> jobs;
    std::vector<int> live;  // indices of successfully parsed jobs
    std::vector<h2j_frame> frames;
    DevBuf d_in, d_arena;
    HostBuf h_in, h_out;
    void* ev[8] = {nullptr};
    double stats[11] = {0};
    // layout of the last run
    size_t zero_bytes = 0, jcoef_base = 0, jcoef_bytes = 0, jstat_base = 0;
    h2j_gpu_batch batch{};

    ~Engine() {
        d_in.release();
        d_arena.release();
        h_in.release();
        h_out.release();
        for (auto& e : ev)
            if (e) h2j_gpu_event_destroy(e);
        if (stream) h2j_gpu_stream_destroy(stream);
        delete pool;
    }

    int fail(const std::string& m) {
        err = m;
        return -1;
    }

    // Upload + run the GPU stages on jobs[live]. stages: 1 recon, 2 +deblock,
    // 3 +sao, 4 +jpeg
    int run_gpu(int stages, bool fetch_jpeg);
};

int Engine::run_gpu(int stages, bool fetch_jpeg) {
    const int nf = static_cast<int>(live.size());
    if (nf == 0) return 0;
    frames.resize(nf);
    size_t ntu = 0, ncoef = 0, nctb = 0, nslice = 0, nsl = 0;
    int max_w = 0, max_h = 0, max_mcu = 0;
    for (int k = 0; k < nf; k++) {
        const FrameJob& j = jobs[live[k]];
        h2j_frame f = j.hdr;
        f.tu = static_cast<uint32_t>(ntu);
        f.ntu = static_cast<uint32_t>(j.tus.size());
        f.coef = static_cast<uint32_t>(ncoef);
        f.ctb = static_cast<uint32_t>(nctb);
        f.slice = static_cast<uint32_t>(nslice);
        f.nslice = static_cast<uint32_t>(j.slices.size());
        f.sl = static_cast<uint32_t>(nsl);
        ntu += j.tus.size();
        ncoef += j.coefs.size();
        nctb += j.ctbs.size();
        nslice += j.slices.size();
        nsl += j.sl.size();
        frames[k] = f;
        max_w = std::max(max_w, f.width);
        max_h = std::max(max_h, f.height);
        max_mcu = std::max(max_mcu, ((f.out_w + 15) >> 4) * ((f.out_h + 15) >> 4));
    }
    // arena layout: [zeroed: maps + jstat][pic][pic2][jcoef]
    size_t off = 0;
    for (int k = 0; k < nf; k++) {
        h2j_frame& f = frames[k];
        f.maps = off;
        off = align_up(off + static_cast<size_t>(f.mw) * f.mh * 2, 256);
    }
    jstat_base = off;
    for (int k = 0; k < nf; k++) {
        frames[k].jstat = off;
        off = align_up(off + sizeof(h2j_jstat), 256);
    }
    zero_bytes = off;
    for (int pass = 0; pass < 2; pass++)
        for (int k = 0; k < nf; k++) {
            h2j_frame& f = frames[k];
            const size_t pel = f.bit_depth > 8 ? 2 : 1;
            const size_t ysz = static_cast<size_t>(f.width) * f.height, csz = ysz / 4;
            f.pic_stride[0] = f.width;
            f.pic_stride[1] = f.pic_stride[2] = f.width / 2;
            f.pic_off[0] = 0;
            f.pic_off[1] = static_cast<int32_t>(ysz);
            f.pic_off[2] = static_cast<int32_t>(ysz + csz);
            if (pass == 0) f.pic = off; else f.pic2 = off;
            off = align_up(off + (ysz + 2 * csz) * pel, 256);
        }
    jcoef_base = off;
    for (int k = 0; k < nf; k++) {
        h2j_frame& f = frames[k];
        f.jcoef = off;
        off = align_up(off + static_cast<size_t>(((f.out_w + 15) >> 4) * ((f.out_h + 15) >> 4)) * 6 * 64 * 2, 256);
    }
    jcoef_bytes = off - jcoef_base;
    const size_t arena_bytes = off;
    // input staging
    const size_t o_frames = 0;
    const size_t o_tus = align_up(o_frames + nf * sizeof(h2j_frame), 256);
    const size_t o_coefs = align_up(o_tus + ntu * sizeof(h2j_tu), 256);
    const size_t o_ctbs = align_up(o_coefs + ncoef * sizeof(h2j_coef), 256);
    const size_t o_slices = align_up(o_ctbs + nctb * sizeof(h2j_ctb), 256);
    const size_t o_sl = align_up(o_slices + nslice * sizeof(h2j_slice), 256);
    const size_t in_bytes = align_up(o_sl + nsl + 16, 256);
    if (!h_in.ensure(in_bytes)) return fail("pinned host allocation failed");
    if (!d_in.ensure(in_bytes)) return fail(std::string("device allocation failed: ") + h2j_gpu_last_error());
    if (!d_arena.ensure(arena_bytes)) return fail(std::string("device allocation failed: ") + h2j_gpu_last_error());
    std::memcpy(h_in.p + o_frames, frames.data(), nf * sizeof(h2j_frame));
    // parallel pack
    std::vector<size_t> bt(nf), bc(nf), bk(nf), bs(nf), bl(nf);
    {
        size_t a = 0, b = 0, c = 0, d = 0, e = 0;
        for (int k = 0; k < nf; k++) {
            const FrameJob& j = jobs[live[k]];
            bt[k] = a; bc[k] = b; bk[k] = c; bs[k] = d; bl[k] = e;
            a += j.tus.size(); b += j.coefs.size(); c += j.ctbs.size(); d += j.slices.size(); e += j.sl.size();
        }
    }
    pool->parallel_for(nf, [&](int k) {
        const FrameJob& j = jobs[live[k]];
        if (!j.tus.empty()) std::memcpy(h_in.p + o_tus + bt[k] * sizeof(h2j_tu), j.tus.data(), j.tus.size() * sizeof(h2j_tu));
        if (!j.coefs.empty()) std::memcpy(h_in.p + o_coefs + bc[k] * sizeof(h2j_coef), j.coefs.data(), j.coefs.size() * sizeof(h2j_coef));
        if (!j.ctbs.empty()) std::memcpy(h_in.p + o_ctbs + bk[k] * sizeof(h2j_ctb), j.ctbs.data(), j.ctbs.size() * sizeof(h2j_ctb));
        if (!j.slices.empty()) std::memcpy(h_in.p + o_slices + bs[k] * sizeof(h2j_slice), j.slices.data(), j.slices.size() * sizeof(h2j_slice));
        if (!j.sl.empty()) std::memcpy(h_in.p + o_sl + bl[k], j.sl.data(), j.sl.size());
    });
    uint8_t* din = static_cast<uint8_t*>(d_in.p);
    batch.nframes = nf;
    batch.max_w = max_w;
    batch.max_h = max_h;
    batch.max_mcu = max_mcu;
    batch.frames = reinterpret_cast<const h2j_frame*>(din + o_frames);
    batch.tus = reinterpret_cast<const h2j_tu*>(din + o_tus);
    batch.coefs = reinterpret_cast<const h2j_coef*>(din + o_coefs);
    batch.ctbs = reinterpret_cast<const h2j_ctb*>(din + o_ctbs);
    batch.slices = reinterpret_cast<const h2j_slice*>(din + o_slices);
    batch.sl = din + o_sl;
    batch.arena = static_cast<uint8_t*>(d_arena.p);
    int r = 0;
    r |= h2j_gpu_event_record(ev[0], stream);
    r |= h2j_gpu_memcpy_h2d(din, h_in.p, in_bytes, stream);
    r |= h2j_gpu_memset(d_arena.p, 0, zero_bytes, stream);
    r |= h2j_gpu_event_record(ev[1], stream);
    if (r) return fail(std::string("upload failed: ") + h2j_gpu_last_error());
    if (h2j_gpu_recon(&batch, stream)) return fail(h2j_gpu_last_error());
    h2j_gpu_event_record(ev[2], stream);
    if (stages >= 2 && h2j_gpu_deblock(&batch, stream)) return fail(h2j_gpu_last_error());
    h2j_gpu_event_record(ev[3], stream);
    if (stages >= 3 && h2j_gpu_sao(&batch, stream)) return fail(h2j_gpu_last_error());
    h2j_gpu_event_record(ev[4], stream);
    if (stages >= 4 && h2j_gpu_jpeg(&batch, stream)) return fail(h2j_gpu_last_error());
    h2j_gpu_event_record(ev[5], stream);
    if (fetch_jpeg) {
        const size_t out_bytes = jcoef_bytes + (zero_bytes - jstat_base);
        if (!h_out.ensure(out_bytes)) return fail("pinned host allocation failed");
        r |= h2j_gpu_memcpy_d2h(h_out.p, static_cast<uint8_t*>(d_arena.p) + jcoef_base, jcoef_bytes, stream);
        r |= h2j_gpu_memcpy_d2h(h_out.p + jcoef_bytes, static_cast<uint8_t*>(d_arena.p) + jstat_base,
                                zero_bytes - jstat_base, stream);
    }
    h2j_gpu_event_record(ev[6], stream);
    if (r) return fail(std::string("download failed: ") + h2j_gpu_last_error());
    if (h2j_gpu_stream_sync(stream)) return fail(std::string("GPU execution failed: ") + h2j_gpu_last_error());
    stats[1] = h2j_gpu_event_elapsed_ms(ev[0], ev[1]);
    stats[2] = h2j_gpu_event_elapsed_ms(ev[1], ev[2]);
    stats[3] = h2j_gpu_event_elapsed_ms(ev[2], ev[3]);
    stats[4] = h2j_gpu_event_elapsed_ms(ev[3], ev[4]);
    stats[5] = h2j_gpu_event_elapsed_ms(ev[4], ev[5]);
    stats[6] = h2j_gpu_event_elapsed_ms(ev[5], ev[6]);
    double bytes = 0;
    for (int k = 0; k < nf; k++) {
        const double S = 1.5 * frames[k].out_w * frames[k].out_h;
        bytes += S * (4.0 + (frames[k].bit_depth > 8 ? 2.0 : 1.0));
    }
    stats[10] = bytes;
    return 0;
}

}  // namespace h2j

using h2j::Engine;

struct h2j_engine {
    Engine e;
};

extern "C" {

const char* h2j_version(void) { return "h2j-mi355x 0.1 (gfx950, HIP)"; }

h2j_engine* h2j_engine_create(int device, int host_threads) {
    if (h2j_gpu_device_count() <= 0) return nullptr;
    if (h2j_gpu_set_device(device) != 0) return nullptr;
    h2j_engine* w = new h2j_engine();
    Engine& e = w->e;
    e.device = device;
    e.stream = h2j_gpu_stream_create();
    if (!e.stream) {
        delete w;
        return nullptr;
    }
    for (auto& ev : e.ev) ev = h2j_gpu_event_create();
    int t = host_threads;
    if (t <= 0) {
        t = static_cast<int>(std::thread::hardware_concurrency());
        if (t > 16) t = 16;
        if (t < 1) t = 1;
    }
    e.pool = new h2j::ThreadPool(t - 1);
    return w;
}

void h2j_engine_destroy(h2j_engine* e) { delete e; }

const char* h2j_engine_error(h2j_engine* e) { return e ? e->e.err.c_str() : "no engine"; }

int h2j_engine_transcode(h2j_engine* w, int n, const uint8_t* const* data, const size_t* sizes, uint8_t* out,
                         size_t out_cap, size_t* out_off, size_t* out_len, int* status) {
    if (!w) return -1;
    Engine& e = w->e;
    if (h2j_gpu_set_device(e.device)) return e.fail(h2j_gpu_last_error());
    const double t0 = h2j::now_ms();
    if (static_cast<int>(e.jobs.size()) < n) e.jobs.resize(n);
    e.pool->parallel_for(n, [&](int i) { h2j::parse_any(data[i], sizes[i], e.jobs[i]); });
    const double t1 = h2j::now_ms();
    e.live.clear();
    for (int i = 0; i < n; i++) {
        status[i] = e.jobs[i].error;
        out_len[i] = 0;
        out_off[i] = 0;
        if (e.jobs[i].error == 0) e.live.push_back(i);
    }
    if (e.run_gpu(4, true)) return -2;
    const double t2 = h2j::now_ms();
    // Huffman + assembly per frame into thread-local vectors, then copy out
    const int nf = static_cast<int>(e.live.size());
    std::vector<std::vector<uint8_t>> jp(nf);
    const uint8_t* jc = e.h_out.p;
    const uint8_t* js = e.h_out.p + e.jcoef_bytes;
    e.pool->parallel_for(nf, [&](int k) {
        const h2j_frame& f = e.frames[k];
        const int16_t* co = reinterpret_cast<const int16_t*>(jc + (f.jcoef - e.jcoef_base));
        const h2j_jstat* st = reinterpret_cast<const h2j_jstat*>(js + (f.jstat - e.jstat_base));
        h2j::jpeg_assemble(co, f.out_w, f.out_h, *st, h2j::kLavcIdent, jp[k]);
    });
    size_t pos = 0;
    int rc = 0;
    for (int k = 0; k < nf; k++) {
        const int i = e.live[k];
        if (pos + jp[k].size() > out_cap) {
            status[i] = -50;
            rc = -3;
            continue;
        }
        std::memcpy(out + pos, jp[k].data(), jp[k].size());
        out_off[i] = pos;
        out_len[i] = jp[k].size();
        pos += jp[k].size();
    }
    const double t3 = h2j::now_ms();
    e.stats[0] = t1 - t0;
    e.stats[7] = t3 - t2;
    e.stats[8] = t3 - t0;
    e.stats[9] = nf;
    if (rc) e.err = "output buffer too small";
    return rc;
}

static int single_job(h2j_engine* w, const uint8_t* data, size_t size) {
    Engine& e = w->e;
    if (h2j_gpu_set_device(e.device)) return e.fail(h2j_gpu_last_error());
    if (e.jobs.empty()) e.jobs.resize(1);
    int r = h2j::parse_any(data, size, e.jobs[0]);
    if (r) return e.fail("parse failed: " + e.jobs[0].message);
    e.live.assign(1, 0);
    return 0;
}

int h2j_engine_decode(h2j_engine* w, const uint8_t* data, size_t size, int stage, uint16_t* planes_out,
                      size_t cap, int* info) {
    if (!w) return -1;
    Engine& e = w->e;
    if (single_job(w, data, size)) return -2;
    const int stages = stage == 1 ? 1 : (stage == 2 ? 2 : 3);
    if (e.run_gpu(stages, false)) return -3;
    const h2j_frame& f = e.frames[0];
    const int w_ = f.out_w, h_ = f.out_h;
    const size_t need = static_cast<size_t>(w_) * h_ * 3 / 2;
    info[0] = w_;
    info[1] = h_;
    info[2] = f.bit_depth;
    if (cap < need) return e.fail("output buffer too small");
    const size_t pel = f.bit_depth > 8 ? 2 : 1;
    const uint64_t base = stage == 0 ? f.pic2 : f.pic;
    const size_t pic_bytes = static_cast<size_t>(f.width) * f.height * 3 / 2 * pel;
    std::vector<uint8_t> tmp(pic_bytes);
    if (h2j_gpu_memcpy_d2h(tmp.data(), static_cast<uint8_t*>(e.d_arena.p) + base, pic_bytes, e.stream) ||
        h2j_gpu_stream_sync(e.stream))
        return e.fail(h2j_gpu_last_error());
    size_t o = 0;
    for (int c = 0; c < 3; c++) {
        const int sh = c ? 1 : 0;
        const int cw = w_ >> sh, ch = h_ >> sh;
        for (int y = 0; y < ch; y++)
            for (int x = 0; x < cw; x++) {
                const size_t idx = static_cast<size_t>(f.pic_off[c]) +
                                   static_cast<size_t>(y + (f.crop_y >> sh)) * f.pic_stride[c] + x + (f.crop_x >> sh);
                planes_out[o++] = pel == 1 ? tmp[idx] : reinterpret_cast<const uint16_t*>(tmp.data())[idx];
            }
    }
    return 0;
}

int h2j_engine_jpeg_coeffs(h2j_engine* w, const uint8_t* data, size_t size, int16_t* out, size_t cap, int* info) {
    if (!w) return -1;
    Engine& e = w->e;
    if (single_job(w, data, size)) return -2;
    if (e.run_gpu(4, true)) return -3;
    const h2j_frame& f = e.frames[0];
    const int nmcu = ((f.out_w + 15) >> 4) * ((f.out_h + 15) >> 4);
    const h2j_jstat* st = reinterpret_cast<const h2j_jstat*>(e.h_out.p + e.jcoef_bytes + (f.jstat - e.jstat_base));
    info[0] = f.out_w;
    info[1] = f.out_h;
    info[2] = st->qscale;
    info[3] = nmcu;
    if (cap < static_cast<size_t>(nmcu) * 384) return e.fail("output buffer too small");
    std::memcpy(out, e.h_out.p + (f.jcoef - e.jcoef_base), static_cast<size_t>(nmcu) * 384 * 2);
    return 0;
}

int h2j_engine_stats(h2j_engine* w, double* out, int n) {
    if (!w) return -1;
    for (int i = 0; i < n && i < 11; i++) out[i] = w->e.stats[i];
    return 0;
}

}  // extern "C"

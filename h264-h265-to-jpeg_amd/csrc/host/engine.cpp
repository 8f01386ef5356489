// Batch engine: host entropy threads -> HBM job records -> HIP pixel and
// JPEG pipeline -> host container assembly.  One engine per process per GPU;
// the IDecoder facade and the C ABI (include/h2j.h) both run on it.
//
// A batch is cut into chunks that flow through two slots (HIP stream +
// device/pinned buffers each), so the host parses chunk c+1 and assembles
// chunk c-1 while the GPU runs chunk c.  Per chunk:
//   1. parse      — pool threads run the H.264/H.265 entropy decoders
//                   (hevc_parser.cpp / h264_parser.cpp) into FrameJobs
//   2. pack + H2D — job records packed into one pinned staging buffer, one copy
//   3. GPU        — K1 recon, K2 deblock, K3 SAO, K4 JPEG forward path,
//                   K5 Huffman tables + entropy-coded payload
//   4. D2H        — per-frame tables (h2j_jstat) and the packed payloads only
//   5. assemble   — pool threads write the JPEG containers (jpeg_writer.cpp)
// This is what the reference does per call inside FFmpeg between
// avcodec_send_packet (/root/reference/src/Decoder.cpp:324) and
// av_write_frame (/root/reference/src/Encoder.cpp:278).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <pthread.h>
#include <sched.h>

#include "affinity.h"
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
    // n workers; cpus: if non-empty, every worker runs on that CPU set (NUMA-local slice)
    explicit ThreadPool(int n, const std::vector<int>& cpus = std::vector<int>()) : stop_(false), gen_(0), pending_(0) {
        for (int i = 0; i < n; i++) workers_.emplace_back([this] { loop(); });
        if (!cpus.empty()) {
            cpu_set_t set;
            CPU_ZERO(&set);
            for (int c : cpus)
                if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &set);
            for (auto& t : workers_)
                if (pthread_setaffinity_np(t.native_handle(), sizeof(set), &set) == 0) pinned_ = true;
        }
    }
    bool pinned() const { return pinned_; }
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
    bool pinned_ = false;
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

// One in-flight chunk: its stream, buffers and layout.
struct Slot {
    void* stream = nullptr;
    // 9: after the stats D2H, 10 / 11: around the in-stream payload D2H, 12 / 13: around the wait for
    // the other slot, 14 / 15: around a second (whole) payload copy
    void* ev[16] = {nullptr};
    size_t pay_pre = 0;        // payload bytes already copied in-stream by enqueue() (estimated, <= h_seg's capacity)
    double px = 0;             // output pixels of the chunk (payload estimate)
    int small_runs = 0;        // consecutive chunks whose payload used < 1/4 of h_seg (shrink after 8)
    size_t small_max = 0;      // the largest payload of that run
    DevBuf d_in, d_arena, d_seg, d_scratch;
    HostBuf h_in, h_js, h_seg;
    std::vector<h2j_frame> frames;
    std::vector<int> live;  // job index of each frame of the chunk
    std::vector<FrameJob>* jobs = nullptr;  // the job set `live` indexes
    h2j_gpu_batch batch{};
    size_t zero_bytes = 0, jcoef_base = 0, jcoef_bytes = 0, jstat_base = 0, jstat_stride = 0;
    int stages = 0;
    bool entropy = false, pending = false;

    void release() {
        d_in.release();
        d_arena.release();
        d_seg.release();
        d_scratch.release();
        h_in.release();
        h_js.release();
        h_seg.release();
        for (auto& e : ev)
            if (e) h2j_gpu_event_destroy(e);
        if (stream) h2j_gpu_stream_destroy(stream);
        stream = nullptr;
    }
};

// stats slots (h2j_engine_stats): times in ms summed over chunks; ST_RECON is K1 only, ST_PREP is K0
// ST_PARSE: submission -> last picture parsed (includes waiting behind the previous batch's parse);
// ST_PARSE_RUN: first -> last picture parsed (the pool's time on this batch)
// ST_D2H_STATS / ST_D2H_PAY: the two parts of ST_D2H (per-picture jstat records; JPEG payloads),
// ST_PAY_BYTES: payload bytes produced, ST_PAY_COPIED: payload bytes moved (the in-stream copy moves
// the pinned buffer's capacity), ST_HOST_GROW: host ms spent growing the pinned payload buffer
// 
enum { ST_PARSE, ST_H2D, ST_RECON, ST_DEBLOCK, ST_SAO, ST_JPEG, ST_D2H, ST_ASSEMBLE, ST_TOTAL, ST_FRAMES, ST_BYTES,
       ST_ENTROPY, ST_PREP, ST_CHUNKS, ST_PACK, ST_PARSE_RUN, ST_D2H_STATS, ST_D2H_PAY, ST_PAY_BYTES, ST_HOST_GROW,
       ST_H2D_BYTES, ST_PAY_COPIED, ST_N };  // ST_PACK: host time packing records into staging

// H.264 pictures with more MB rows than this are reconstructed by several K1 workgroups
constexpr int kK1BandRows = 68;

// upper bound of one block's entropy-coded size (code lengths <= 16, values <= 16 bits)
constexpr size_t kSegBytesPerBlock = 272;

struct ChunkTime {
    int frames = 0;
    double k1_ms = 0, kernels_ms = 0;  // K1 launch; K0..K5 (HIP events on the chunk's stream)
};

// A submitted batch (h2j_engine_submit; h2j_engine_transcode is submit + wait).
struct Batch {
    int64_t ticket = 0;
    int n = 0;
    const uint8_t* const* data = nullptr;  // caller-owned until the batch is waited for
    const size_t* sizes = nullptr;
    uint8_t* out = nullptr;
    size_t out_cap = 0;
    size_t* out_off = nullptr;
    size_t* out_len = nullptr;
    int* status = nullptr;
    std::vector<int> bounds;                   // parse chunks: index ranges
    std::vector<int> chunk_of;
    std::unique_ptr<std::atomic<int>[]> left;  // pictures of each parse chunk still being parsed
    int jobset = -1;                           // Engine::jobsets slot the batch parses into
    bool parsed = false, done = false;
    int rc = 0;
    double t0 = 0, t_parse0 = 0, t_parsed = 0;
    // results handed to the caller by h2j_engine_wait (per ticket: a later batch that finishes
    // before this one is waited for does not overwrite them)
    double stats[ST_N] = {0};
    std::vector<ChunkTime> chunk_log;
    std::vector<std::string> msg;  // parse messages of the failed pictures
    std::string err;
};

struct Engine {
    int device = 0;
    ThreadPool* pool = nullptr;
    HostPlan plan;  // host threads / NUMA placement of the pool
    std::string err;
    std::vector<FrameJob> jobs;  // single-picture entry points (decode / jpeg_coeffs)
    // Asynchronous batches: a parser thread runs the pool over batch after batch, a driver thread
    // runs each batch's GPU chunks and JPEG assembly, so one batch's GPU tail overlaps the next
    // batch's entropy decoding.  At most two batches hold a job set at a time.
    std::mutex amu;
    std::condition_variable acv;
    std::deque<Batch*> parse_q, gpu_q;
    std::vector<std::unique_ptr<Batch>> batches;  // submitted and not yet waited for
    std::vector<FrameJob> jobsets[2];
    bool jobset_busy[2] = {false, false};
    int64_t next_ticket = 1;
    int active = 0;  // submitted batches not done
    bool stop = false;
    std::thread parser, driver;
    std::mutex pool_mu;  // held by whoever runs a parallel_for on the pool
    // results of the last batch a caller waited for (h2j_engine_wait copies them under amu; they
    // stay valid until the next wait returns)
    double last_stats[ST_N] = {0};
    std::vector<int> last_status;          // per-picture status
    std::vector<std::string> last_msg;     // ... and the parse messages of its failed pictures
    std::vector<ChunkTime> last_chunk_log;  // its chunks (h2j_engine_chunk_times)
    std::vector<ChunkTime> chunk_log;       // chunks of the batch being driven (driver thread)
    std::string derr;                       // error of the batch being driven (driver thread)
    Slot slot[2];
    double stats[ST_N] = {0};  // working stats of the batch being driven
    double slot_hbm_budget = 64e9;  // per slot; shared with the other engines on the device
    double pay_per_px = 0;          // JPEG payload bytes per output pixel, running estimate (both slots)
    bool strict_reference = false;  // H2J_STRICT_REFERENCE=1: fail where the reference returns false

    ~Engine() {
        {
            std::unique_lock<std::mutex> lk(amu);
            acv.wait(lk, [&] { return active == 0; });
            stop = true;
        }
        acv.notify_all();
        if (parser.joinable()) parser.join();
        if (driver.joinable()) driver.join();
        slot[0].release();
        slot[1].release();
        delete pool;
    }

    // run f(i), i < n, on the pool if no one else is using it (the parser), else on this thread
    void par(int n, const std::function<void(int)>& f) {
        if (pool_mu.try_lock()) {
            pool->parallel_for(n, f);
            pool_mu.unlock();
        } else {
            for (int i = 0; i < n; i++) f(i);
        }
    }
    void start_threads();
    void parse_loop();
    void drive_loop();
    int run_batch(Batch& b);
    // wait until no batch is in flight (the single-picture entry points use slot 0 directly)
    void quiesce() {
        std::unique_lock<std::mutex> lk(amu);
        acv.wait(lk, [&] { return active == 0; });
    }

    // the driver thread reports into the batch it drives (a caller may be reading `err`)
    int fail(const std::string& m) {
        if (driver.joinable() && std::this_thread::get_id() == driver.get_id()) derr = m;
        else err = m;
        return -1;
    }
    // an enqueue that fails after its first async operation: wait for what was queued on the
    // slot's stream, so the staging / device buffers are idle before anyone reuses or frees them
    int drain_fail(Slot& s, const std::string& m) {
        h2j_gpu_stream_sync(s.stream);
        return fail(m);
    }

    // Lay out, pack and enqueue the GPU work of jobs[live] on slot s.
    // stages: 1 recon, 2 +deblock, 3 +sao, 4 +jpeg forward path; entropy: +K5.
    // pool_free: the thread pool may be used for packing (not busy parsing).
    // `after`: the other slot, when its kernels are still in flight -- this slot's kernels start once
    // they have finished (its copies and the host's assembly still overlap them)
    int enqueue(Slot& s, int stages, bool entropy, bool pool_free = true, const Slot* after = nullptr);  // s.jobs must be set
    // Wait for slot s and copy its payloads down (entropy chunks).
    int sync(Slot& s);
};

int Engine::enqueue(Slot& s, int stages, bool entropy, bool pool_free, const Slot* after) {
    const int nf = static_cast<int>(s.live.size());
    s.stages = stages;
    s.entropy = entropy;
    s.pending = false;
    if (nf == 0) return 0;
    s.frames.resize(nf);
    size_t ntu = 0, ncoef = 0, nctb = 0, nslice = 0, nsl = 0, nblk = 0;
    int max_w = 0, max_h = 0, max_mcu = 0, max_ntu = 0, max_ctbs = 0;
    const std::vector<FrameJob>& jobs = *s.jobs;
    for (int k = 0; k < nf; k++) {
        const FrameJob& j = jobs[s.live[k]];
        max_ntu = std::max(max_ntu, static_cast<int>(j.tus.size()));
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
        // H.264 K1: pictures taller than 1080p run on one workgroup per 16 MB rows
        // (a single 16-wave workgroup would walk 5+ rows per wave)
        // (MBAFF frames run on one workgroup: their K1 / deblocking walk macroblock pairs)
        f.k1bands = (f.codec == H2J_CODEC_H264 && f.ctb_h > kK1BandRows && !f.mbaff) ? (f.ctb_h + 15) / 16 : 1;
        f.xline = 0;
        s.frames[k] = f;
        max_w = std::max(max_w, f.width);
        if (f.codec == H2J_CODEC_HEVC) max_ctbs = std::max(max_ctbs, f.ctb_w * f.ctb_h);
        max_h = std::max(max_h, f.height);
        const int mcu = ((f.out_w + 15) >> 4) * ((f.out_h + 15) >> 4);
        max_mcu = std::max(max_mcu, mcu);
        nblk += static_cast<size_t>(mcu) * 6;
    }
    // arena layout: [zeroed: maps + CTB TU ranges + jstat][pic][pic2][jcoef][res][aux]
    size_t off = 0;
    for (int k = 0; k < nf; k++) {
        h2j_frame& f = s.frames[k];
        f.maps = off;
        off = align_up(off + static_cast<size_t>(f.mw) * f.mh * 2, 256);
        f.ctbrng = off;
        off = align_up(off + static_cast<size_t>(f.ctb_w) * f.ctb_h * 16, 256);  // [first, first chroma, end, -]
    }
    s.jstat_base = off;
    s.jstat_stride = align_up(sizeof(h2j_jstat), 256);
    for (int k = 0; k < nf; k++) {
        s.frames[k].jstat = off;
        off += s.jstat_stride;
    }
    s.zero_bytes = off;
    for (int pass = 0; pass < 2; pass++)
        for (int k = 0; k < nf; k++) {
            h2j_frame& f = s.frames[k];
            const size_t pel = f.bit_depth > 8 ? 2 : 1;
            const size_t ysz = static_cast<size_t>(f.width) * f.height, csz = ysz / 4;
            f.pic_stride[0] = f.width;
            f.pic_stride[1] = f.pic_stride[2] = f.width / 2;
            f.pic_off[0] = 0;
            f.pic_off[1] = static_cast<int32_t>(ysz);
            f.pic_off[2] = static_cast<int32_t>(ysz + csz);
            if (pass == 1 && (f.codec != H2J_CODEC_HEVC || !f.sao_enabled)) {
                f.pic2 = f.pic;  // no SAO: the deblocked picture is the decoded picture (K3 skips it)
                continue;
            }
            if (pass == 0) f.pic = off; else f.pic2 = off;
            off = align_up(off + (ysz + 2 * csz) * pel, 256);
        }
    s.jcoef_base = off;
    for (int k = 0; k < nf; k++) {  // dense int16 plane (inspection) or the JPEG symbol tiles
        h2j_frame& f = s.frames[k];
        f.jcoef = off;
        const size_t blocks = static_cast<size_t>(((f.out_w + 15) >> 4) * ((f.out_h + 15) >> 4)) * 6;
        off = align_up(off + std::max(blocks * 64 * 2, (blocks + 255) / 256 * static_cast<size_t>(H2J_JTILE_BYTES)), 256);
    }
    s.jcoef_bytes = off - s.jcoef_base;
    for (int k = 0; k < nf; k++) {
        h2j_frame& f = s.frames[k];
        const size_t ysz = static_cast<size_t>(f.width) * f.height;
        // HEVC residual planes are tiled by K1 quadrant (include/h2j_gpu.h h2j_res_elems: whole
        // tiles, a little more than the picture); H.264 keeps the picture's raster layout
        const size_t res_elems = f.codec == H2J_CODEC_HEVC
                                     ? static_cast<size_t>(h2j_res_elems(f.width, f.height, f.log2ctb))
                                     : ysz + ysz / 2;
        f.res = off;
        off = align_up(off + res_elems * 2, 256);
        f.aux = off;
        off = align_up(off + static_cast<size_t>(f.ntu) * 8, 256);
        if (f.k1bands > 1) {  // per band boundary: K1 1 luma + 2 chroma rows, K2 4 luma + 2x2 chroma rows (uint16)
            f.xline = off;   // K1's 8-row bands and K2's 16-row bands use it one after the other
            const size_t k2b = static_cast<size_t>(f.k1bands - 1) * 6 * f.width * 2;
            const size_t k1b = static_cast<size_t>((f.ctb_h + 7) / 8 - 1) * 2 * f.width * 2;
            off = align_up(off + std::max(k1b, k2b), 256);
        }
    }
    const size_t arena_bytes = off;
    // input staging
    const size_t o_frames = 0;
    const size_t o_tus = align_up(o_frames + nf * sizeof(h2j_frame), 256);
    const size_t o_coefs = align_up(o_tus + ntu * sizeof(h2j_tu), 256);
    const size_t o_ctbs = align_up(o_coefs + ncoef * sizeof(h2j_coef), 256);
    const size_t o_slices = align_up(o_ctbs + nctb * sizeof(h2j_ctb), 256);
    const size_t o_sl = align_up(o_slices + nslice * sizeof(h2j_slice), 256);
    // H.264 K1 workgroup map: banded pictures first (their long chains start early), bands in order,
    // then the others by transform-block count, most first (the dispatcher hands workgroups out in
    // map order: the heaviest pictures start in the first round, not in the launch's tail)
    // Banded pictures band-major (every picture's band 0, then every band 1, ...): a band waits on
    // the band above, and picture-major order had each picture's lower bands holding workgroup
    // slots while they waited (a batch of 4K H.264 pictures ran at a fraction of the GPU).  A band
    // still follows the band above it in the map, so it never waits on one not yet dispatched.
    std::vector<uint32_t> k1map;
    {
        int maxb = 0;
        for (int k = 0; k < nf; k++)
            if (s.frames[k].codec == H2J_CODEC_H264 && s.frames[k].k1bands > 1) maxb = std::max(maxb, static_cast<int>(s.frames[k].k1bands));
        for (int bnd = 0; bnd < maxb; bnd++)
            for (int k = 0; k < nf; k++) {
                const h2j_frame& f = s.frames[k];
                if (f.codec != H2J_CODEC_H264 || f.k1bands <= 1 || bnd >= static_cast<int>(f.k1bands)) continue;
                k1map.push_back((static_cast<uint32_t>(k) << 8) | static_cast<uint32_t>(bnd));
            }
    }
    // the same for h2j_k1_recon_h264's 8-wave workgroups: bands of 8 rows (16-row bands took two
    // row rounds each, so a band below started a whole row time after the band above)
    std::vector<uint32_t> k1map8;
    {
        int maxb = 0;
        for (int k = 0; k < nf; k++)
            if (s.frames[k].codec == H2J_CODEC_H264 && s.frames[k].k1bands > 1) maxb = std::max(maxb, (s.frames[k].ctb_h + 7) / 8);
        for (int bnd = 0; bnd < maxb; bnd++)
            for (int k = 0; k < nf; k++) {
                const h2j_frame& f = s.frames[k];
                if (f.codec != H2J_CODEC_H264 || f.k1bands <= 1 || bnd >= (f.ctb_h + 7) / 8) continue;
                k1map8.push_back((static_cast<uint32_t>(k) << 8) | static_cast<uint32_t>(bnd));
            }
    }
    {
        std::vector<std::pair<uint32_t, uint32_t>> un;
        for (int k = 0; k < nf; k++) {
            const h2j_frame& f = s.frames[k];
            if (f.codec == H2J_CODEC_H264 && f.k1bands <= 1) un.emplace_back(f.ntu, static_cast<uint32_t>(k));
        }
        std::stable_sort(un.begin(), un.end(), [](const std::pair<uint32_t, uint32_t>& a, const std::pair<uint32_t, uint32_t>& b) {
                return a.first > b.first;
            });
        for (const auto& x : un) {
            k1map.push_back(x.second << 8);
            k1map8.push_back(x.second << 8);
        }
    }
    // mixed-batch K1 map (h2j_k1_recon_any): every HEVC picture and H.264 band, tallest first so
    // the longest chains start first; bands of one picture stay in order
    std::vector<uint32_t> k1all;
    {
        std::vector<std::pair<int, uint32_t>> e;
        for (int k = 0; k < nf; k++) {
            const h2j_frame& f = s.frames[k];
            if (f.codec != H2J_CODEC_HEVC) continue;
            const int rows = f.ctb_h << (f.log2ctb - 4);  // in 16-sample rows
            if (rows > kK1BandRows) {  // taller than 1088: a 16-wave workgroup per component group
                e.emplace_back(-2000 - rows, (3u << 30) | (static_cast<uint32_t>(k) << 8) | 0u);
                e.emplace_back(-2000 - rows, (3u << 30) | (static_cast<uint32_t>(k) << 8) | 1u);
            } else {
                e.emplace_back(-rows, (1u << 31) | (static_cast<uint32_t>(k) << 8));
            }
        }
        for (uint32_t m : k1map) {
            const h2j_frame& f = s.frames[m >> 8];
            e.emplace_back(-std::min(f.ctb_h, 16) - (f.k1bands > 1 ? 1000 : 0), m);
        }
        std::stable_sort(e.begin(), e.end(),
                         [](const std::pair<int, uint32_t>& a, const std::pair<int, uint32_t>& b) { return a.first < b.first; });
        for (const auto& x : e) k1all.push_back(x.second);
    }
    std::vector<uint32_t> k1hevc;
    for (uint32_t m : k1all)
        if (m & 0x80000000u) k1hevc.push_back(m);
    // K3 SAO map: the HEVC pictures with SAO, most CTBs first, cut into CTB-count classes (a picture
    // joins the current class while it has more than half the class's CTBs; the last class takes
    // the rest), one launch each, so no class pays for the largest picture's grid width
    std::vector<uint32_t> saomap;
    int sao_groups = 0, sao_first[H2J_SAO_GROUPS] = {}, sao_count[H2J_SAO_GROUPS] = {}, sao_ctbs[H2J_SAO_GROUPS] = {};
    {
        std::vector<std::pair<int, uint32_t>> e;
        for (int k = 0; k < nf; k++) {
            const h2j_frame& f = s.frames[k];
            if (f.codec == H2J_CODEC_HEVC && f.pic2 != f.pic) e.emplace_back(f.ctb_w * f.ctb_h, static_cast<uint32_t>(k));
        }
        std::stable_sort(e.begin(), e.end(),
                         [](const std::pair<int, uint32_t>& a, const std::pair<int, uint32_t>& b) { return a.first > b.first; });
        for (size_t i = 0; i < e.size(); i++) {
            const bool same = sao_groups > 0 && (sao_groups == H2J_SAO_GROUPS || 2 * e[i].first > sao_ctbs[sao_groups - 1]);
            if (!same) {
                sao_first[sao_groups] = static_cast<int>(i);
                sao_ctbs[sao_groups] = e[i].first;
                sao_groups++;
            }
            sao_count[sao_groups - 1]++;
            saomap.push_back(e[i].second);
        }
    }
    const size_t o_map = align_up(o_sl + nsl + 16, 256);
    const size_t o_all = align_up(o_map + k1map.size() * 4 + 16, 256);
    const size_t o_sao = align_up(o_all + k1all.size() * 4 + 16, 256);
    const size_t o_map8 = align_up(o_sao + saomap.size() * 4 + 16, 256);
    const size_t o_hev = align_up(o_map8 + k1map8.size() * 4 + 16, 256);
    const size_t in_bytes = align_up(o_hev + k1hevc.size() * 4 + 16, 256);
    if (!s.h_in.ensure(in_bytes)) return fail("pinned host allocation failed");
    if (!s.d_in.ensure(in_bytes)) return fail(std::string("device allocation failed: ") + h2j_gpu_last_error());
    if (!s.d_arena.ensure(arena_bytes)) return fail(std::string("device allocation failed: ") + h2j_gpu_last_error());
    const int tiles = (max_mcu * 6 + 255) / 256;
    const size_t seg_cap = nblk * kSegBytesPerBlock + 16 * static_cast<size_t>(nf);
    if (entropy) {
        if (!s.d_seg.ensure(seg_cap)) return fail(std::string("device allocation failed: ") + h2j_gpu_last_error());
        if (!s.d_scratch.ensure(static_cast<size_t>(nf) * tiles * 4 + 256))
            return fail(std::string("device allocation failed: ") + h2j_gpu_last_error());
        if (!s.h_js.ensure(static_cast<size_t>(nf) * s.jstat_stride + 256)) return fail("pinned host allocation failed");
    }
    std::memcpy(s.h_in.p + o_frames, s.frames.data(), nf * sizeof(h2j_frame));
    if (!k1map.empty()) std::memcpy(s.h_in.p + o_map, k1map.data(), k1map.size() * 4);
    if (!k1all.empty()) std::memcpy(s.h_in.p + o_all, k1all.data(), k1all.size() * 4);
    if (!saomap.empty()) std::memcpy(s.h_in.p + o_sao, saomap.data(), saomap.size() * 4);
    if (!k1map8.empty()) std::memcpy(s.h_in.p + o_map8, k1map8.data(), k1map8.size() * 4);
    if (!k1hevc.empty()) std::memcpy(s.h_in.p + o_hev, k1hevc.data(), k1hevc.size() * 4);
    std::vector<size_t> bt(nf), bc(nf), bk(nf), bs(nf), bl(nf);
    {
        size_t a = 0, b = 0, c = 0, d = 0, e = 0;
        for (int k = 0; k < nf; k++) {
            const FrameJob& j = jobs[s.live[k]];
            bt[k] = a; bc[k] = b; bk[k] = c; bs[k] = d; bl[k] = e;
            a += j.tus.size(); b += j.coefs.size(); c += j.ctbs.size(); d += j.slices.size(); e += j.sl.size();
        }
    }
    uint8_t* hin = s.h_in.p;
    auto pack = [&](int k) {
        const FrameJob& j = jobs[s.live[k]];
        if (!j.tus.empty()) std::memcpy(hin + o_tus + bt[k] * sizeof(h2j_tu), j.tus.data(), j.tus.size() * sizeof(h2j_tu));
        if (!j.coefs.empty()) std::memcpy(hin + o_coefs + bc[k] * sizeof(h2j_coef), j.coefs.data(), j.coefs.size() * sizeof(h2j_coef));
        if (!j.ctbs.empty()) std::memcpy(hin + o_ctbs + bk[k] * sizeof(h2j_ctb), j.ctbs.data(), j.ctbs.size() * sizeof(h2j_ctb));
        if (!j.slices.empty()) std::memcpy(hin + o_slices + bs[k] * sizeof(h2j_slice), j.slices.data(), j.slices.size() * sizeof(h2j_slice));
        if (!j.sl.empty()) std::memcpy(hin + o_sl + bl[k], j.sl.data(), j.sl.size());
    };
    const double tp = now_ms();
    if (pool_free) par(nf, pack);
    else for (int k = 0; k < nf; k++) pack(k);
    stats[ST_PACK] += now_ms() - tp;
    uint8_t* din = static_cast<uint8_t*>(s.d_in.p);
    h2j_gpu_batch& b = s.batch;
    b.nframes = nf;
    b.max_w = max_w;
    b.max_h = max_h;
    b.max_mcu = max_mcu;
    b.max_ntu = max_ntu;
    b.max_ctbs = max_ctbs;
    b.has_hevc = 0;
    b.has_h264 = 0;
    b.has_mbaff = 0;
    b.h264_pels = 0;
    for (int k = 0; k < nf; k++) {
        const h2j_frame& fk = s.frames[k];
        if (fk.codec == H2J_CODEC_HEVC) b.has_hevc = 1;
        if (fk.codec != H2J_CODEC_H264) continue;
        b.has_h264 = 1;
        if (fk.mbaff) b.has_mbaff = 1;
        else b.h264_pels |= fk.bit_depth == 8 ? 1 : 2;
    }
    b.frames = reinterpret_cast<const h2j_frame*>(din + o_frames);
    b.tus = reinterpret_cast<const h2j_tu*>(din + o_tus);
    b.coefs = reinterpret_cast<const h2j_coef*>(din + o_coefs);
    b.ctbs = reinterpret_cast<const h2j_ctb*>(din + o_ctbs);
    b.slices = reinterpret_cast<const h2j_slice*>(din + o_slices);
    b.sl = din + o_sl;
    b.k1map = reinterpret_cast<const uint32_t*>(din + o_map);
    b.k1wgs = static_cast<int32_t>(k1map.size());
    b.k1all = reinterpret_cast<const uint32_t*>(din + o_all);
    b.k1all_n = static_cast<int32_t>(k1all.size());
    b.k1map8 = reinterpret_cast<const uint32_t*>(din + o_map8);
    b.k1wgs8 = static_cast<int32_t>(k1map8.size());
    b.k1hevc = reinterpret_cast<const uint32_t*>(din + o_hev);
    b.k1hevc_n = static_cast<int32_t>(k1hevc.size());
    b.sao_map = reinterpret_cast<const uint32_t*>(din + o_sao);
    b.sao_groups = sao_groups;
    for (int g = 0; g < H2J_SAO_GROUPS; g++) {
        b.sao_first[g] = sao_first[g];
        b.sao_count[g] = sao_count[g];
        b.sao_ctbs[g] = sao_ctbs[g];
    }
    b.hevc_pels = 0;
    for (int k = 0; k < nf; k++)
        if (s.frames[k].codec == H2J_CODEC_HEVC) b.hevc_pels |= (s.frames[k].bit_depth > 8 || s.frames[k].bit_depth_c > 8) ? 2 : 1;
    b.arena = static_cast<uint8_t*>(s.d_arena.p);
    b.jpeg_dense = entropy ? 0 : 1;
    {  // pictures whose MB variances K4a sums (K3 sums the others'; no K4a launch when none is left)
        int k4a = 0;
        for (int k = 0; k < nf; k++) k4a += h2j_sao_folds_variance(s.frames[k]) ? 0 : 1;
        b.k4a_frames = k4a;
    }
    b.seg = entropy ? static_cast<uint8_t*>(s.d_seg.p) : nullptr;
    b.seg_cap = entropy ? seg_cap : 0;
    b.seg_total = entropy ? static_cast<uint64_t*>(s.d_scratch.p) : nullptr;
    b.tile_bits = entropy ? reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(s.d_scratch.p) + 256) : nullptr;
    void* st = s.stream;
    int r = 0;
    r |= h2j_gpu_event_record(s.ev[0], st);
    r |= h2j_gpu_memcpy_h2d(din, hin, in_bytes, st);
    r |= h2j_gpu_event_record(s.ev[12], st);
    stats[ST_H2D_BYTES] += static_cast<double>(in_bytes);
    // two GPU sub-chunks of one parsed range (4K batches, mixed batches past the slot's HBM budget)
    // would otherwise run their kernels side by side: the GPU is not the bound (the host entropy
    // threads are), and concurrent launches inflated every stage's event time and rocprof duration
    // (r05: 4K K4b 1.14 ms and the arena fill 1.18 ms per 256 pictures, 0.004 / 0.037 ms alone)
    if (after && after->pending) r |= h2j_gpu_stream_wait_event(st, after->ev[6]);
    r |= h2j_gpu_event_record(s.ev[13], st);
    r |= h2j_gpu_memset(s.d_arena.p, 0, s.zero_bytes, st);
    r |= h2j_gpu_event_record(s.ev[1], st);
    if (r) return drain_fail(s, std::string("upload failed: ") + h2j_gpu_last_error());
    if (h2j_gpu_prep(&b, st)) return drain_fail(s, h2j_gpu_last_error());
    h2j_gpu_event_record(s.ev[8], st);
    if (h2j_gpu_predict(&b, st)) return drain_fail(s, h2j_gpu_last_error());
    h2j_gpu_event_record(s.ev[2], st);
    if (stages >= 2 && h2j_gpu_deblock(&b, st)) return drain_fail(s, h2j_gpu_last_error());
    h2j_gpu_event_record(s.ev[3], st);
    if (stages >= 3 && h2j_gpu_sao(&b, st)) return drain_fail(s, h2j_gpu_last_error());
    h2j_gpu_event_record(s.ev[4], st);
    if (stages >= 4 && h2j_gpu_jpeg(&b, st)) return drain_fail(s, h2j_gpu_last_error());
    h2j_gpu_event_record(s.ev[5], st);
    if (entropy && h2j_gpu_entropy(&b, st)) return drain_fail(s, h2j_gpu_last_error());
    h2j_gpu_event_record(s.ev[6], st);
    if (entropy) {
        r |= h2j_gpu_memcpy_d2h(s.h_js.p, s.d_scratch.p, 8, st);  // seg_total
        r |= h2j_gpu_memcpy_d2h(s.h_js.p + 256, static_cast<uint8_t*>(s.d_arena.p) + s.jstat_base,
                                static_cast<size_t>(nf) * s.jstat_stride, st);
        if (r) return drain_fail(s, std::string("download failed: ") + h2j_gpu_last_error());
    }
    h2j_gpu_event_record(s.ev[9], st);
    // the payloads follow in the same stream, sized by the pinned buffer (1.25x the largest total
    // seen): no host round trip between the kernels and the copy.  r04/r05 enqueued the copy in
    // sync() once the host had read the total: at 4K its interval measured 40-78 ms per step for
    // 121 MB against 4 ms for the bare copy (tools/d2h_probe: 30 GB/s pinned) -- the submitting
    // driver thread waited for CPU behind the 16 entropy threads (profiles/r05_4k_d2h.md).  A
    // total above the capacity (first chunks, growth) is copied again whole in sync().
    if (s.small_runs >= 8) {  // the slot's last chunk has been assembled: h_seg is free to go
        const double tg = now_ms();
        const size_t keep = s.small_max + s.small_max / 4 + 16;
        s.h_seg.release();
        if (!s.h_seg.ensure(keep)) return fail("pinned host allocation failed");
        stats[ST_HOST_GROW] += now_ms() - tg;
        s.small_runs = 0;
    }
    s.pay_pre = 0;
    s.px = 0;
    for (int k = 0; k < nf; k++) s.px += static_cast<double>(s.frames[k].out_w) * s.frames[k].out_h;
    if (entropy && s.h_seg.cap > 0) {
        // the copy is sized by the engine's payload-per-pixel estimate (1.3x, 4 KB
        // granules), not by the buffer's high-water mark: a small chunk after a 4K one moves its own
        // few MB, not the 4K chunk's 150 MB
        size_t want = seg_cap;
        if (pay_per_px > 0) want = (static_cast<size_t>(1.3 * pay_per_px * s.px) + 65536 + 4095) & ~static_cast<size_t>(4095);
        s.pay_pre = std::min(std::min(s.h_seg.cap, seg_cap), want);
        h2j_gpu_event_record(s.ev[10], st);
        if (h2j_gpu_memcpy_d2h(s.h_seg.p, s.d_seg.p, s.pay_pre, st))
            return drain_fail(s, std::string("download failed: ") + h2j_gpu_last_error());
        h2j_gpu_event_record(s.ev[11], st);
    }
    s.pending = true;
    double bytes = 0;
    for (int k = 0; k < nf; k++) {
        const double S = 1.5 * s.frames[k].out_w * s.frames[k].out_h;
        bytes += S * (4.0 + (s.frames[k].bit_depth > 8 ? 2.0 : 1.0));
    }
    stats[ST_BYTES] += bytes;
    return 0;
}

int Engine::sync(Slot& s) {
    if (!s.pending) return 0;
    s.pending = false;
    if (h2j_gpu_stream_sync(s.stream)) return fail(std::string("GPU execution failed: ") + h2j_gpu_last_error());
    bool pay_late = false;
    if (s.entropy) {
        uint64_t total = 0;
        std::memcpy(&total, s.h_js.p, 8);
        stats[ST_PAY_BYTES] += static_cast<double>(total);
        if (s.px > 0) {  // payload per pixel: a running mean, never below the last chunk's
            const double ratio = static_cast<double>(total) / s.px;
            pay_per_px = pay_per_px > 0 ? std::max(ratio, 0.7 * pay_per_px + 0.3 * ratio) : ratio;
        }
        stats[ST_PAY_COPIED] += static_cast<double>(s.pay_pre);  // the in-stream copy, used or not
        if (total > s.pay_pre) {  // not (all) copied in-stream: grow with headroom, copy it whole
            const double tg = now_ms();
            if (!s.h_seg.ensure(total + total / 4 + 16)) return fail("pinned host allocation failed");
            stats[ST_HOST_GROW] += now_ms() - tg;
            stats[ST_PAY_COPIED] += static_cast<double>(total);
            pay_late = true;
            h2j_gpu_event_record(s.ev[14], s.stream);
            if (h2j_gpu_memcpy_d2h(s.h_seg.p, s.d_seg.p, total, s.stream))
                return fail(std::string("download failed: ") + h2j_gpu_last_error());
            h2j_gpu_event_record(s.ev[15], s.stream);
        }
        // the pinned buffer shrinks after 8 chunks in a row that used less than a quarter of it
        if (total * 4 < s.h_seg.cap) {
            s.small_max = s.small_runs ? std::max(s.small_max, static_cast<size_t>(total)) : static_cast<size_t>(total);
            s.small_runs++;
        } else {
            s.small_runs = 0;
        }
    }
    if (h2j_gpu_event_record(s.ev[7], s.stream) || h2j_gpu_stream_sync(s.stream))
        return fail(std::string("download failed: ") + h2j_gpu_last_error());
    // the H2D copy alone; the arena fill (after any wait for the other slot's kernels) counts with K0
    stats[ST_H2D] += h2j_gpu_event_elapsed_ms(s.ev[0], s.ev[12]);
    stats[ST_PREP] += h2j_gpu_event_elapsed_ms(s.ev[13], s.ev[8]);
    stats[ST_RECON] += h2j_gpu_event_elapsed_ms(s.ev[8], s.ev[2]);
    stats[ST_CHUNKS] += 1;
    stats[ST_DEBLOCK] += h2j_gpu_event_elapsed_ms(s.ev[2], s.ev[3]);
    stats[ST_SAO] += h2j_gpu_event_elapsed_ms(s.ev[3], s.ev[4]);
    stats[ST_JPEG] += h2j_gpu_event_elapsed_ms(s.ev[4], s.ev[5]);
    stats[ST_ENTROPY] += h2j_gpu_event_elapsed_ms(s.ev[5], s.ev[6]);
    // copies only (the payload copy is enqueued once the host has read the sizes)
    const double d2h_stats = h2j_gpu_event_elapsed_ms(s.ev[6], s.ev[9]);
    // both payload copies when the in-stream one fell short (the second one's events had
    // overwritten the first's)
    const double d2h_pay = (s.entropy && s.pay_pre ? h2j_gpu_event_elapsed_ms(s.ev[10], s.ev[11]) : 0.0) +
                           (pay_late ? h2j_gpu_event_elapsed_ms(s.ev[14], s.ev[15]) : 0.0);
    stats[ST_D2H] += d2h_stats + d2h_pay;
    stats[ST_D2H_STATS] += d2h_stats;
    stats[ST_D2H_PAY] += d2h_pay;
    ChunkTime ct;
    ct.frames = static_cast<int>(s.live.size());
    ct.k1_ms = h2j_gpu_event_elapsed_ms(s.ev[8], s.ev[2]);
    ct.kernels_ms = h2j_gpu_event_elapsed_ms(s.ev[13], s.ev[6]);
    chunk_log.push_back(ct);
    return 0;
}

// Chunk boundaries: chunks large enough to fill the GPU (K1 runs one
// workgroup per picture), small enough that parse / GPU / assembly overlap;
// the last quarter is split into shrinking chunks so that the GPU work left
// after the last picture is parsed (the pipeline's tail) is short.
std::vector<int> chunk_plan(int n) {
    int chunk = n >= 512 ? 256 : n;
    const char* e = std::getenv("H2J_CHUNK");
    if (e && std::atoi(e) > 0) chunk = std::atoi(e);
    chunk = std::max(1, chunk);
    const char* tail = std::getenv("H2J_TAIL");  // "0": no shrinking tail chunks
    const bool shrink = !(tail && tail[0] == '0');
    const char* tmin = std::getenv("H2J_TAIL_MIN");  // smallest tail chunk (default 128: 256,256,256,128,128 for 1024)
    const int tail_min = tmin && std::atoi(tmin) > 0 ? std::atoi(tmin) : 128;
    std::vector<int> starts;
    int i = 0;
    while (i < n) {
        starts.push_back(i);
        int c = chunk;
        const int left = n - i;
        if (shrink && left <= chunk && left > tail_min && chunk >= 128) c = left / 2;  // tail: halve
        i += std::min(c, left);
    }
    starts.push_back(n);
    return starts;
}

// Throughput plan (asynchronous batches): one parse chunk of up to 1024 pictures (K1 runs up to
// four pictures per workgroup on launches that large); the GPU tail of a batch is hidden behind
// the next batch's entropy decoding instead of being cut into shrinking chunks.
std::vector<int> chunk_plan_throughput(int n) {
    int chunk = 1024;
    const char* e = std::getenv("H2J_CHUNK_ASYNC");
    if (e && std::atoi(e) > 0) chunk = std::atoi(e);
    std::vector<int> starts;
    for (int i = 0; i < n; i += chunk) starts.push_back(i);
    starts.push_back(n);
    return starts;
}

// GPU sub-chunks of a parsed range are bounded by an HBM estimate per slot (pictures, residual,
// JPEG symbol tiles, payload pool: ~20 B per luma sample at 8 bits) and by 1024 pictures.
constexpr double kSlotHbmBudget = 64e9;  // at most, per slot (two slots per engine)
constexpr int kMaxGpuChunk = 1024;
static double hbm_estimate(const FrameJob& j) {
    const double px = static_cast<double>(j.hdr.width) * j.hdr.height;
    return px * (j.hdr.bit_depth > 8 ? 24.0 : 20.0) + (1 << 20);
}

void Engine::start_threads() {
    std::lock_guard<std::mutex> g(amu);
    if (parser.joinable()) return;
    parser = std::thread([this] { parse_loop(); });
    driver = std::thread([this] { drive_loop(); });
}

void Engine::parse_loop() {
    for (;;) {
        Batch* b = nullptr;
        {
            std::unique_lock<std::mutex> lk(amu);
            acv.wait(lk, [&] { return stop || !parse_q.empty(); });
            if (parse_q.empty()) return;
            b = parse_q.front();
            parse_q.pop_front();
            acv.wait(lk, [&] { return !jobset_busy[0] || !jobset_busy[1]; });
            b->jobset = jobset_busy[0] ? 1 : 0;
            jobset_busy[b->jobset] = true;
        }
        b->t_parse0 = now_ms();
        std::vector<FrameJob>& jobs = jobsets[b->jobset];
        if (static_cast<int>(jobs.size()) < b->n) jobs.resize(static_cast<size_t>(b->n));
        // batches smaller than the thread pool (a lone IDecoder call): pictures with several
        // independent slices / WPP rows / tiles parse them on several threads
        const int slice_threads = std::max(1, (pool->size() + 1) / std::max(1, b->n));
        // inside each chunk the largest bitstreams start first (the threads then finish a chunk
        // together instead of idling behind one large picture); chunks keep their order
        std::vector<int> order(static_cast<size_t>(b->n));
        for (int i = 0; i < b->n; i++) order[i] = i;
        for (size_t c = 0; c + 1 < b->bounds.size(); c++)
            std::stable_sort(order.begin() + b->bounds[c], order.begin() + b->bounds[c + 1],
                             [&](int x, int y) { return b->sizes[x] > b->sizes[y]; });
        {
            std::lock_guard<std::mutex> g(pool_mu);
            pool->parallel_for(b->n, [&](int k) {
                const int i = order[static_cast<size_t>(k)];
                jobs[i].threads = slice_threads;
                parse_any(b->data[i], b->sizes[i], jobs[i]);
                if (b->left[b->chunk_of[i]].fetch_sub(1) == 1) {
                    std::lock_guard<std::mutex> g2(amu);
                    acv.notify_all();
                }
            });
        }
        std::lock_guard<std::mutex> g(amu);
        b->t_parsed = now_ms();
        b->parsed = true;
        acv.notify_all();
    }
}

void Engine::drive_loop() {
    h2j_gpu_set_device(device);  // HIP's current device is per thread
    for (;;) {
        Batch* b = nullptr;
        {
            std::unique_lock<std::mutex> lk(amu);
            acv.wait(lk, [&] { return stop || !gpu_q.empty(); });
            if (gpu_q.empty()) return;
            b = gpu_q.front();
            gpu_q.pop_front();
        }
        derr.clear();
        const int rc = run_batch(*b);
        std::unique_lock<std::mutex> lk(amu);
        acv.wait(lk, [&] { return b->parsed; });  // a failed batch may still be parsing
        std::vector<FrameJob>* jobs = b->jobset >= 0 ? &jobsets[b->jobset] : nullptr;
        stats[ST_PARSE] = b->t_parsed > 0 ? b->t_parsed - b->t0 : 0;
        stats[ST_PARSE_RUN] = b->t_parsed > 0 ? b->t_parsed - b->t_parse0 : 0;
        stats[ST_TOTAL] = now_ms() - b->t0;
        std::memcpy(b->stats, stats, sizeof(stats));
        b->chunk_log = chunk_log;
        b->err = derr;
        b->msg.assign(static_cast<size_t>(b->n), std::string());
        if (jobs)
            for (int i = 0; i < b->n; i++)
                if (b->status[i] != 0 && (*jobs)[i].error != 0) b->msg[i] = (*jobs)[i].message;
        if (b->jobset >= 0) jobset_busy[b->jobset] = false;
        b->rc = rc;
        b->done = true;
        active--;
        acv.notify_all();
    }
}

// The GPU side of one batch (driver thread): as parse chunks complete, their pictures go to the
// two slots in GPU sub-chunks (HBM budget); slot c+1 is enqueued before slot c is assembled, so
// the GPU runs one sub-chunk while the host writes the JPEGs of the previous one.
int Engine::run_batch(Batch& b) {
    for (auto& v : stats) v = 0;
    chunk_log.clear();
    const int nchunks = static_cast<int>(b.bounds.size()) - 1;
    if (b.n == 0 || nchunks <= 0) return 0;
    size_t pos = 0;
    int rc = 0;
    int* status = b.status;
    auto assemble = [&](Slot& s) -> int {
        if (sync(s)) return -2;
        const double ta = now_ms();
        const int nf = static_cast<int>(s.live.size());
        const uint8_t* js = s.h_js.p + 256;
        std::vector<size_t> sz(nf);
        auto size_of = [&](int k) {
            const h2j_jstat* st = reinterpret_cast<const h2j_jstat*>(js + k * s.jstat_stride);
            sz[k] = st->seg_off == ~0ull ? 0 : jpeg_container_size(*st, s.h_seg.p + st->seg_off, kLavcIdent);
        };
        par(nf, size_of);
        std::vector<size_t> at(nf);
        for (int k = 0; k < nf; k++) {
            const int i = s.live[k];
            const h2j_jstat* stk = reinterpret_cast<const h2j_jstat*>(js + k * s.jstat_stride);
            if (stk->dev_error) {  // a device-side failure (e.g. a K1 band hand-off timed out)
                status[i] = -52;
                rc = -3;
                at[k] = ~static_cast<size_t>(0);
                continue;
            }
            if (!sz[k]) {
                status[i] = -51;  // payload pool overflow
                rc = -3;
                at[k] = ~static_cast<size_t>(0);
                continue;
            }
            if (pos + sz[k] > b.out_cap) {
                status[i] = -50;
                rc = -3;
                at[k] = ~static_cast<size_t>(0);
                continue;
            }
            at[k] = pos;
            b.out_off[i] = pos;
            b.out_len[i] = sz[k];
            pos += sz[k];
        }
        auto write = [&](int k) {
            if (at[k] == ~static_cast<size_t>(0)) return;
            const h2j_jstat* st = reinterpret_cast<const h2j_jstat*>(js + k * s.jstat_stride);
            const h2j_frame& f = s.frames[k];
            jpeg_write_container(*st, s.h_seg.p + st->seg_off, f.out_w, f.out_h, kLavcIdent, b.out + at[k]);
        };
        par(nf, write);
        stats[ST_ASSEMBLE] += now_ms() - ta;
        stats[ST_FRAMES] += nf;
        return 0;
    };
    int fail = 0, sc = 0;
    for (int c = 0; c < nchunks && !fail; c++) {
        {
            std::unique_lock<std::mutex> lk(amu);
            acv.wait(lk, [&] { return b.left[c].load() == 0; });
        }
        std::vector<FrameJob>& jobs = jobsets[b.jobset];
        int i = b.bounds[c];
        const int end = b.bounds[c + 1];
        // equal shares of the range's HBM estimate, as few as the budget allows (uneven splits
        // leave small, latency-bound launches behind)
        double total = 0;
        for (int k = i; k < end; k++) total += hbm_estimate(jobs[k]);
        const double budget = slot_hbm_budget;
        const int parts = std::max(static_cast<int>(std::ceil(total / budget)),
                                   (end - i + kMaxGpuChunk - 1) / kMaxGpuChunk);
        const double share = total / std::max(1, parts);
        while (i < end && !fail) {
            int j = i;
            double est = 0;
            while (j < end && j - i < kMaxGpuChunk) {
                const double cst = hbm_estimate(jobs[j]);
                if (j > i && (est + cst > budget || est + cst / 2 > share)) break;
                est += cst;
                j++;
            }
            Slot& s = slot[sc & 1];
            if (s.pending && assemble(s)) { fail = 1; break; }
            s.live.clear();
            s.jobs = &jobs;
            for (int k = i; k < j; k++) {
                if (strict_reference && jobs[k].error == 0 && jobs[k].reorder_delay) {
                    // the reference sends one packet and never flushes: avcodec_receive_frame gives
                    // EAGAIN for a stream with output reordering and H265ToJpeg returns false
                    // (/root/reference/src/Decoder.cpp:324, 342-360)
                    jobs[k].error = -7;
                    jobs[k].message = "decoder delay: no picture before a flush (H2J_STRICT_REFERENCE)";
                }
                if (strict_reference && jobs[k].error == 0 && jobs[k].field_pair) {
                    // one packet holds one field: FFmpeg waits for the second field and the
                    // reference returns false (/root/reference/src/Decoder.cpp:324, 342-360)
                    jobs[k].error = -3;
                    jobs[k].message = "field picture (PAFF): no frame from one field (H2J_STRICT_REFERENCE)";
                }
                status[k] = jobs[k].error;
                if (jobs[k].error == 0) s.live.push_back(k);
            }
            Slot& prev = slot[(sc + 1) & 1];
            if (enqueue(s, 4, true, true, &prev)) { fail = 1; break; }
            if (sc > 0 && prev.pending && assemble(prev)) { fail = 1; break; }
            sc++;
            i = j;
        }
    }
    for (int k = 0; k < 2 && !fail; k++) {
        Slot& s = slot[(sc + k) & 1];
        if (s.pending && assemble(s)) fail = 1;
    }
    if (fail) {
        for (auto& s : slot)
            if (s.pending) sync(s);
        return -2;
    }
    if (rc) derr = "output buffer too small or payload pool overflow";
    return rc;
}

}  // namespace h2j

using h2j::Engine;
using h2j::Slot;

struct h2j_engine {
    Engine e;
};

extern "C" {

const char* h2j_version(void) { return "h2j-mi355x 0.2 (gfx950, HIP)"; }

h2j_engine* h2j_engine_create(int device, int host_threads) {
    if (h2j_gpu_device_count() <= 0) return nullptr;
    if (h2j_gpu_set_device(device) != 0) return nullptr;
    h2j_engine* w = new h2j_engine();
    Engine& e = w->e;
    e.device = device;
    for (auto& s : e.slot) {
        s.stream = h2j_gpu_stream_create();
        if (!s.stream) {
            delete w;
            return nullptr;
        }
        for (auto& ev : s.ev) ev = h2j_gpu_event_create();
    }
    // host pool: NUMA-local to the device, sized by the CPU mask / cgroup quota (affinity.h)
    std::vector<int> nodes;
    const int ndev = h2j_gpu_device_count();
    for (int i = 0; i < ndev; i++) {
        char bus[64] = {0};
        nodes.push_back(h2j_gpu_pci_bus_id(i, bus, sizeof(bus)) == 0 ? h2j::pci_numa_node(bus) : -1);
    }
    const int node = device >= 0 && device < ndev ? nodes[device] : -1;
    e.plan = h2j::plan_host(device, nodes, h2j::process_cpus(), h2j::node_cpus(node), h2j::cgroup_cpu_quota(),
                            host_threads > 0 ? host_threads : 0, host_threads < 0 ? -host_threads : 1);
    e.pool = new h2j::ThreadPool(e.plan.threads - 1, e.plan.cpus);
    // HBM per slot: 64 GB at most, and the device's memory split between the two slots of every
    // engine of this process on the device (host_threads = -k: k engines dealt over the devices)
    const int k = host_threads < 0 ? -host_threads : 1;
    const int per_dev = std::max(1, k / std::max(1, ndev) + (device < k % std::max(1, ndev) ? 1 : 0));
    size_t free_b = 0, total_b = 0;
    double budget = h2j::kSlotHbmBudget;
    if (h2j_gpu_mem_info(&free_b, &total_b) == 0 && total_b > 0)
        budget = std::min(budget, 0.8 * static_cast<double>(total_b) / (2.0 * per_dev));
    e.slot_hbm_budget = budget;
    const char* strict = std::getenv("H2J_STRICT_REFERENCE");
    e.strict_reference = strict && strict[0] == '1';
    return w;
}

void h2j_engine_destroy(h2j_engine* e) { delete e; }

const char* h2j_engine_error(h2j_engine* e) { return e ? e->e.err.c_str() : "no engine"; }

// submit one batch; latency: the synchronous plan (small tail chunks), else the throughput plan
static int64_t submit_batch(h2j_engine* w, int n, const uint8_t* const* data, const size_t* sizes, uint8_t* out,
                            size_t out_cap, size_t* out_off, size_t* out_len, int* status, bool latency) {
    Engine& e = w->e;
    std::unique_ptr<h2j::Batch> b(new h2j::Batch());
    b->n = n;
    b->data = data;
    b->sizes = sizes;
    b->out = out;
    b->out_cap = out_cap;
    b->out_off = out_off;
    b->out_len = out_len;
    b->status = status;
    for (int i = 0; i < n; i++) {
        out_len[i] = 0;
        out_off[i] = 0;
        status[i] = 0;
    }
    b->bounds = latency ? h2j::chunk_plan(n) : h2j::chunk_plan_throughput(n);
    const int nchunks = static_cast<int>(b->bounds.size()) - 1;
    b->chunk_of.assign(static_cast<size_t>(n), 0);
    for (int c = 0; c < nchunks; c++)
        for (int i = b->bounds[c]; i < b->bounds[c + 1]; i++) b->chunk_of[i] = c;
    b->left.reset(new std::atomic<int>[std::max(1, nchunks)]);
    for (int c = 0; c < nchunks; c++) b->left[c] = b->bounds[c + 1] - b->bounds[c];
    e.start_threads();
    std::lock_guard<std::mutex> g(e.amu);
    b->ticket = e.next_ticket++;
    b->t0 = h2j::now_ms();
    const int64_t t = b->ticket;
    e.active++;
    e.parse_q.push_back(b.get());
    e.gpu_q.push_back(b.get());
    e.batches.push_back(std::move(b));
    e.acv.notify_all();
    return t;
}

int64_t h2j_engine_submit(h2j_engine* w, int n, const uint8_t* const* data, const size_t* sizes, uint8_t* out,
                          size_t out_cap, size_t* out_off, size_t* out_len, int* status) {
    if (!w || n < 0) return -1;
    return submit_batch(w, n, data, sizes, out, out_cap, out_off, out_len, status, false);
}

int h2j_engine_wait(h2j_engine* w, int64_t ticket) {
    if (!w) return -1;
    Engine& e = w->e;
    std::unique_lock<std::mutex> lk(e.amu);
    auto it = std::find_if(e.batches.begin(), e.batches.end(),
                           [&](const std::unique_ptr<h2j::Batch>& b) { return b->ticket == ticket; });
    if (it == e.batches.end()) return -1;
    h2j::Batch* b = it->get();
    e.acv.wait(lk, [&] { return b->done; });
    const int rc = b->rc;
    std::memcpy(e.last_stats, b->stats, sizeof(b->stats));
    e.last_chunk_log.swap(b->chunk_log);
    e.last_status.assign(b->status, b->status + b->n);
    e.last_msg.swap(b->msg);
    if (rc) e.err = b->err;
    e.batches.erase(it);
    return rc;
}

int h2j_engine_transcode(h2j_engine* w, int n, const uint8_t* const* data, const size_t* sizes, uint8_t* out,
                         size_t out_cap, size_t* out_off, size_t* out_len, int* status) {
    if (!w) return -1;
    const int64_t t = submit_batch(w, n, data, sizes, out, out_cap, out_off, out_len, status, true);
    return h2j_engine_wait(w, t);
}

static int single_job(h2j_engine* w, const uint8_t* data, size_t size) {
    Engine& e = w->e;
    e.quiesce();
    if (h2j_gpu_set_device(e.device)) return e.fail(h2j_gpu_last_error());
    if (e.jobs.empty()) e.jobs.resize(1);
    e.jobs[0].threads = e.pool->size() + 1;  // independent slices on several threads
    int r = h2j::parse_any(data, size, e.jobs[0]);
    if (r) return e.fail("parse failed: " + e.jobs[0].message);
    e.slot[0].live.assign(1, 0);
    e.slot[0].jobs = &e.jobs;
    return 0;
}

// copy picture k of slot s (after sync) out as uint16 cropped planes
static int copy_planes(Engine& e, Slot& s, int k, int stage, uint16_t* planes_out, size_t cap, int* info) {
    const h2j_frame& f = s.frames[k];
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
    if (h2j_gpu_memcpy_d2h(tmp.data(), static_cast<uint8_t*>(s.d_arena.p) + base, pic_bytes, s.stream) ||
        h2j_gpu_stream_sync(s.stream))
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

int h2j_engine_decode(h2j_engine* w, const uint8_t* data, size_t size, int stage, uint16_t* planes_out,
                      size_t cap, int* info) {
    if (!w) return -1;
    Engine& e = w->e;
    if (single_job(w, data, size)) return -2;
    const int stages = stage == 1 ? 1 : (stage == 2 ? 2 : 3);
    Slot& s = e.slot[0];
    if (e.enqueue(s, stages, false) || e.sync(s)) return -3;
    return copy_planes(e, s, 0, stage, planes_out, cap, info);
}

int h2j_engine_decode_batch(h2j_engine* w, int n, const uint8_t* const* data, const size_t* sizes, int stage, int pick,
                            uint16_t* planes_out, size_t cap, int* info) {
    if (!w || n <= 0 || pick < 0 || pick >= n) return -1;
    Engine& e = w->e;
    e.quiesce();
    if (h2j_gpu_set_device(e.device)) return e.fail(h2j_gpu_last_error());
    e.jobs.resize(n);
    std::vector<int> rc(n, 0);
    e.par(n, [&](int i) {
        e.jobs[i].threads = 1;
        rc[i] = h2j::parse_any(data[i], sizes[i], e.jobs[i]);
    });
    for (int i = 0; i < n; i++)
        if (rc[i]) {
            e.fail("parse failed (picture " + std::to_string(i) + "): " + e.jobs[i].message);
            return -2;
        }
    Slot& s = e.slot[0];
    s.live.resize(n);
    for (int i = 0; i < n; i++) s.live[i] = i;
    s.jobs = &e.jobs;
    const int stages = stage == 1 ? 1 : (stage == 2 ? 2 : 3);
    if (e.enqueue(s, stages, false) || e.sync(s)) return -3;
    return copy_planes(e, s, pick, stage, planes_out, cap, info);
}

int h2j_engine_jpeg_coeffs(h2j_engine* w, const uint8_t* data, size_t size, int16_t* out, size_t cap, int* info) {
    if (!w) return -1;
    Engine& e = w->e;
    if (single_job(w, data, size)) return -2;
    Slot& s = e.slot[0];
    if (e.enqueue(s, 4, false) || e.sync(s)) return -3;
    const h2j_frame& f = s.frames[0];
    const int nmcu = ((f.out_w + 15) >> 4) * ((f.out_h + 15) >> 4);
    h2j_jstat st;
    if (cap < static_cast<size_t>(nmcu) * 384) return e.fail("output buffer too small");
    if (h2j_gpu_memcpy_d2h(&st, static_cast<uint8_t*>(s.d_arena.p) + f.jstat, sizeof(st), s.stream) ||
        h2j_gpu_memcpy_d2h(out, static_cast<uint8_t*>(s.d_arena.p) + f.jcoef, static_cast<size_t>(nmcu) * 384 * 2,
                           s.stream) ||
        h2j_gpu_stream_sync(s.stream))
        return e.fail(h2j_gpu_last_error());
    info[0] = f.out_w;
    info[1] = f.out_h;
    info[2] = st.qscale;
    info[3] = nmcu;
    return 0;
}

int h2j_engine_host_info(h2j_engine* w, int* out, int n) {
    if (!w) return -1;
    const Engine& e = w->e;
    const int v[4] = {e.pool->size() + 1, e.plan.numa_node, e.pool->pinned() ? static_cast<int>(e.plan.cpus.size()) : 0,
                      e.plan.cpus.empty() ? -1 : e.plan.cpus[0]};
    for (int i = 0; i < n && i < 4; i++) out[i] = v[i];
    return 0;
}

const char* h2j_engine_frame_error(h2j_engine* w, int i) {
    if (!w) return "";
    std::lock_guard<std::mutex> g(w->e.amu);
    if (i < 0 || i >= static_cast<int>(w->e.last_status.size())) return "";
    switch (w->e.last_status[i]) {
    case 0: return "";
    case -50: return "output buffer too small";
    case -51: return "JPEG payload pool overflow";
    case -52: return "device-side failure (a K1 / deblocking progress wait timed out)";
    default: {
        // copied under the lock into a per-thread buffer: h2j_engine_wait on another thread may
        // replace last_msg (and free its strings) as soon as the lock is released
        static thread_local std::string buf;
        buf = i < static_cast<int>(w->e.last_msg.size()) ? w->e.last_msg[i] : std::string();
        return buf.c_str();
    }
    }
}

int h2j_device_count(void) { return h2j_gpu_device_count(); }

int h2j_engine_chunk_times(h2j_engine* w, double* out, int max_chunks) {
    if (!w) return -1;
    std::lock_guard<std::mutex> g(w->e.amu);
    const auto& log = w->e.last_chunk_log;
    const int n = static_cast<int>(log.size());
    for (int i = 0; i < n && i < max_chunks; i++) {
        out[3 * i] = log[i].frames;
        out[3 * i + 1] = log[i].k1_ms;
        out[3 * i + 2] = log[i].kernels_ms;
    }
    return n;
}

int h2j_engine_stats(h2j_engine* w, double* out, int n) {
    if (!w) return -1;
    std::lock_guard<std::mutex> g(w->e.amu);
    for (int i = 0; i < n && i < h2j::ST_N; i++) out[i] = w->e.last_stats[i];
    return 0;
}

}  // extern "C"

// IDecoder facade — drop-in for the reference's Decoder
// (/root/reference/src/Decoder.cpp:39-53 getInstance, :115-361 H265ToJpeg)
// and Encoder (/root/reference/src/Encoder.cpp:104-362).  Same contract:
// borrowed C-string paths, fresh instance per getInstance(), false + a LOG
// line on any failure, output written with fopen("wb+") + fwrite.
// Differences (documented in DESIGN.md): no probe-decode, no fixed 2 MiB
// output buffer (the reference's writeCallback has no bounds check,
// src/Encoder.cpp:29), decoder-delay streams are handled (the first picture
// is decoded directly), 10-bit input is converted with
// v8 = min(255, (v + 2) >> 2) instead of producing a corrupted JPEG.
#include <algorithm>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "IDecoder.h"
#include "h2j.h"

void LOG(const char* format, ...) {
    char log[1024] = {0};
    va_list ap;
    va_start(ap, format);
    vsnprintf(log, sizeof(log), format, ap);
    va_end(ap);
    time_t ts;
    time(&ts);
    struct tm tmv;
    localtime_r(&ts, &tmv);  // the reference's localtime() is not thread-safe
    char now[64];
    strftime(now, sizeof(now), "%Y-%m-%d %H:%M:%S", &tmv);
    printf("%s | %s\n", now, log);
}

namespace {

// One engine per visible GPU (H2J_ENGINES overrides the count; engine i runs on device
// i % device count); IDecoder instances are cheap handles.  Concurrent H265ToJpeg calls are
// batched: callers queue their bitstreams, and whichever caller finds engines idle takes
// everything queued, splits it over the idle engines (longest-processing-time first by
// bitstream bytes, the host entropy cost) and runs the parts as h2j_engine_transcode batches
// side by side (host entropy decoding fans out over each engine's thread pool, each GPU sees
// one launch per stage), then hands every caller its JPEG.  A lone caller runs a batch of one;
// a JVM calling through JNI from many threads keeps every GPU of the node busy.
struct Request {
    const uint8_t* data = nullptr;
    size_t size = 0;
    std::vector<uint8_t> jpeg;
    int status = 0;
    std::string error;
    bool done = false;
};

struct EngineSlot {
    h2j_engine* e = nullptr;
    bool busy = false;
};

std::mutex g_mu;
std::condition_variable g_cv;
std::deque<Request*> g_queue;
std::vector<EngineSlot> g_engines;
bool g_engines_init = false;

// create the engines (caller holds g_mu); none when no HIP device is visible
void init_engines_locked() {
    if (g_engines_init) return;
    g_engines_init = true;
    const int ndev = h2j_device_count();
    if (ndev <= 0) return;
    int n = ndev;
    if (const char* env = getenv("H2J_ENGINES")) {
        const int v = atoi(env);
        if (v > 0 && v <= 64) n = v;
    }
    for (int i = 0; i < n; i++) {
        // split the host threads between the engines (each creates a pool of that size)
        h2j_engine* e = h2j_engine_create(i % ndev, -n);
        if (e) {
            EngineSlot slot;
            slot.e = e;
            g_engines.push_back(slot);
        }
    }
}

// LPT partition of `work` into k parts by bitstream bytes (each part keeps queue order)
std::vector<std::vector<Request*>> split_lpt(const std::vector<Request*>& work, int k) {
    std::vector<int> idx(work.size());
    for (size_t i = 0; i < idx.size(); i++) idx[i] = static_cast<int>(i);
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return work[a]->size > work[b]->size; });
    std::vector<size_t> load(static_cast<size_t>(k), 0);
    std::vector<int> part(work.size());
    for (int i : idx) {
        const int m = static_cast<int>(std::min_element(load.begin(), load.end()) - load.begin());
        part[i] = m;
        load[m] += work[i]->size + 1;
    }
    std::vector<std::vector<Request*>> out(static_cast<size_t>(k));
    for (size_t i = 0; i < work.size(); i++) out[part[i]].push_back(work[i]);
    return out;
}

// run one batch (caller holds no lock); fills jpeg / status / error of each request
void run_batch(h2j_engine* e, std::vector<Request*>& batch) {
    const int n = static_cast<int>(batch.size());
    if (n == 0) return;
    std::vector<const uint8_t*> ptrs(n);
    std::vector<size_t> sizes(n), off(n), len(n);
    std::vector<int> status(n);
    size_t cap = 8u << 20;
    for (int i = 0; i < n; i++) {
        ptrs[i] = batch[i]->data;
        sizes[i] = batch[i]->size;
        cap += batch[i]->size * 4 + (2u << 20);
    }
    std::vector<uint8_t> out;
    int r = -1;
    for (int attempt = 0; attempt < 3; attempt++) {
        out.resize(cap);
        r = h2j_engine_transcode(e, n, ptrs.data(), sizes.data(), out.data(), cap, off.data(), len.data(),
                                 status.data());
        bool small = false;
        for (int i = 0; i < n; i++) small = small || status[i] == -50;
        if (!small) break;
        cap *= 4;
    }
    for (int i = 0; i < n; i++) {
        Request* q = batch[i];
        q->status = status[i];
        if (r != 0 && status[i] == 0) q->status = r;
        if (q->status == 0) {
            q->jpeg.assign(out.begin() + static_cast<long>(off[i]), out.begin() + static_cast<long>(off[i] + len[i]));
        } else {
            const char* m = status[i] != 0 ? h2j_engine_frame_error(e, i) : "";
            q->error = (m && *m) ? m : h2j_engine_error(e);
        }
    }
}

// transcode pictures through the shared, batching engines (all of `reqs` join the same queue,
// so a caller's own batch runs together with whatever else is queued)
void transcode_shared_many(const std::vector<Request*>& reqs) {
    std::unique_lock<std::mutex> lk(g_mu);
    init_engines_locked();
    if (g_engines.empty()) {
        for (Request* q : reqs) {
            q->status = -1;
            q->error = "no HIP device available: the MI355X pipeline cannot run";
            q->done = true;
        }
        return;
    }
    for (Request* r : reqs) g_queue.push_back(r);
    auto all_done = [&] {
        for (Request* r : reqs)
            if (!r->done) return false;
        return true;
    };
    while (!all_done()) {
        std::vector<int> idle;
        for (size_t i = 0; i < g_engines.size(); i++)
            if (!g_engines[i].busy) idle.push_back(static_cast<int>(i));
        if (idle.empty() || g_queue.empty()) {
            g_cv.wait(lk);
            continue;
        }
        std::vector<Request*> work(g_queue.begin(), g_queue.end());
        g_queue.clear();
        const int k = static_cast<int>(std::min(idle.size(), work.size()));
        std::vector<std::vector<Request*>> parts = split_lpt(work, k);
        for (int j = 0; j < k; j++) g_engines[idle[j]].busy = true;
        lk.unlock();
        std::vector<std::thread> helpers;
        for (int j = 1; j < k; j++)
            helpers.emplace_back([&, j] { run_batch(g_engines[idle[j]].e, parts[j]); });
        run_batch(g_engines[idle[0]].e, parts[0]);
        for (auto& t : helpers) t.join();
        lk.lock();
        for (Request* q : work) q->done = true;
        for (int j = 0; j < k; j++) g_engines[idle[j]].busy = false;
        g_cv.notify_all();
    }
}

bool transcode_shared(Request& req) {
    transcode_shared_many(std::vector<Request*>{&req});
    return req.status == 0;
}

bool read_file(const char* path, std::vector<uint8_t>& buf) {
    FILE* f = fopen(path, "rb");
    if (!f) return false;
    if (fseek(f, 0, SEEK_END) != 0) { fclose(f); return false; }
    long n = ftell(f);
    if (n < 0) { fclose(f); return false; }
    rewind(f);
    buf.resize(static_cast<size_t>(n));
    size_t got = n ? fread(buf.data(), 1, static_cast<size_t>(n), f) : 0;
    fclose(f);
    return got == static_cast<size_t>(n);
}

class Decoder : public IDecoder {
public:
    Decoder() { LOG("%s", __PRETTY_FUNCTION__); }
    ~Decoder() override = default;
    bool H265ToJpeg(const char* inputFilePath, const char* outputFilePath) override;
};

bool Decoder::H265ToJpeg(const char* const in, const char* const out) {
    if (in == nullptr || out == nullptr || strlen(in) == 0 || strlen(out) == 0) {
        LOG("input or output path is empty: input:%s, output:%s", in ? in : "(null)", out ? out : "(null)");
        return false;
    }
    std::vector<uint8_t> data;
    if (!read_file(in, data)) {
        LOG("cannot open input file: %s", in);
        return false;
    }
    Request req;
    req.data = data.data();
    req.size = data.size();
    if (!transcode_shared(req)) {
        LOG("transcode failed (%d): %s", req.status, req.error.c_str());
        return false;
    }
    const std::vector<uint8_t>& jpeg = req.jpeg;
    FILE* f = fopen(out, "wb+");
    if (!f) {
        LOG("failed to encode Yuv to Jpeg: cannot open %s", out);
        return false;
    }
    size_t w = fwrite(jpeg.data(), 1, jpeg.size(), f);
    fclose(f);
    if (w != jpeg.size()) {
        LOG("failed to write Jpeg file %s", out);
        return false;
    }
    LOG("saved Jpeg data to file %s", out);
    return true;
}

}  // namespace

std::shared_ptr<IDecoder> IDecoder::getInstance() { return std::make_shared<Decoder>(); }

// ---- in-memory and batch entry points beside IDecoder

extern "C" int h2j_h265_to_jpeg_mem(const uint8_t* data, size_t size, uint8_t** jpeg, size_t* jpeg_len) {
    if (!jpeg || !jpeg_len) return -1;
    *jpeg = nullptr;
    *jpeg_len = 0;
    if (!data || size == 0) return -1;
    Request req;
    req.data = data;
    req.size = size;
    if (!transcode_shared(req)) {
        LOG("transcode failed (%d): %s", req.status, req.error.c_str());
        return req.status ? req.status : -1;
    }
    uint8_t* p = static_cast<uint8_t*>(malloc(req.jpeg.size()));
    if (!p) return -1;
    std::memcpy(p, req.jpeg.data(), req.jpeg.size());
    *jpeg = p;
    *jpeg_len = req.jpeg.size();
    return 0;
}

extern "C" void h2j_free(void* p) { free(p); }

extern "C" int h2j_h265_to_jpeg_batch(const char* const* in_paths, const char* const* out_paths, int n, int* ok) {
    if (n <= 0 || !in_paths || !out_paths) return 0;
    std::vector<std::vector<uint8_t>> data(static_cast<size_t>(n));
    std::vector<Request> reqs(static_cast<size_t>(n));
    std::vector<Request*> live;
    for (int i = 0; i < n; i++) {
        if (ok) ok[i] = 0;
        const char* in = in_paths[i];
        const char* out = out_paths[i];
        if (!in || !out || !*in || !*out) {
            LOG("input or output path is empty: input:%s, output:%s", in ? in : "(null)", out ? out : "(null)");
            continue;
        }
        if (!read_file(in, data[i])) {
            LOG("cannot open input file: %s", in);
            continue;
        }
        reqs[i].data = data[i].data();
        reqs[i].size = data[i].size();
        live.push_back(&reqs[i]);
    }
    if (!live.empty()) transcode_shared_many(live);
    int good = 0;
    for (int i = 0; i < n; i++) {
        const Request& q = reqs[i];
        if (!q.done) continue;
        if (q.status != 0) {
            LOG("transcode failed (%d) for %s: %s", q.status, in_paths[i], q.error.c_str());
            continue;
        }
        FILE* f = fopen(out_paths[i], "wb+");
        if (!f) {
            LOG("failed to encode Yuv to Jpeg: cannot open %s", out_paths[i]);
            continue;
        }
        const size_t w = fwrite(q.jpeg.data(), 1, q.jpeg.size(), f);
        fclose(f);
        if (w != q.jpeg.size()) {
            LOG("failed to write Jpeg file %s", out_paths[i]);
            continue;
        }
        if (ok) ok[i] = 1;
        good++;
    }
    return good;
}

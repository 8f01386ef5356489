// H.264 intra entropy decoding on the host (placeholder until the H.264
// path lands): reports the stream as unsupported.
#include "job.h"

namespace h2j {
int h264_parse_picture(const uint8_t*, size_t, FrameJob& job) {
    job.clear();
    job.error = -101;
    job.message = "H.264 path not built yet";
    return -101;
}
}  // namespace h2j

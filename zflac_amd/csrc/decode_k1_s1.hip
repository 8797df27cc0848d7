// decode_k1_s1.hip -- two-pass stereo decode, 16-bit containers, pass S1 (decode.inc, LAY_S1):
// channel 1, decorrelated with channel 0 read back from the scratch rows, interleaved output.
#include "decode.inc"

namespace zflac {
hipError_t launch_decode_k1_s1(const DecodeArgs& a, uint32_t max_frames, hipStream_t st) {
    return launch_decode_layout<1, LAY_S1>(a, max_frames, st);
}
}  // namespace zflac

// decode_k1_s0.hip -- two-pass stereo decode, 16-bit containers, pass S0 (decode.inc, LAY_S0):
// channel 0 of 64 frames per wave into the per-frame scratch rows, and where channel 1 starts.
#include "decode.inc"

namespace zflac {
hipError_t launch_decode_k1_s0(const DecodeArgs& a, uint32_t max_frames, hipStream_t st) {
    return launch_decode_layout<1, LAY_S0>(a, max_frames, st);
}
}  // namespace zflac

// decode_k2.hip -- decode kernels for SampleType container kind 2 (i32).
#include "decode.inc"

namespace zflac {
hipError_t launch_decode_k2(const DecodeArgs& a, uint32_t max_frames, hipStream_t st) {
    return launch_decode_kind<2>(a, max_frames, st);
}
}  // namespace zflac

// decode_k0.hip -- decode kernels for SampleType container kind 0 (i8).
#include "decode.inc"

namespace zflac {
hipError_t launch_decode_k0(const DecodeArgs& a, uint32_t max_frames, hipStream_t st) {
    return launch_decode_kind<0>(a, max_frames, st);
}
}  // namespace zflac

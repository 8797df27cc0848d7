// decode_k1.hip -- decode kernels for SampleType container kind 1 (i16).
#include "decode.inc"

namespace zflac {
hipError_t launch_decode_k1(const DecodeArgs& a, uint32_t max_frames, hipStream_t st) {
    return launch_decode_kind<1>(a, max_frames, st);
}
}  // namespace zflac

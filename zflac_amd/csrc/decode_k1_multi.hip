// decode_k1_multi.hip -- decode kernel for SampleType container kind 1 (i16), multi layout.
// One translation unit per (container, layout) so the instantiations compile in parallel.
#include "decode.inc"

namespace zflac {
hipError_t launch_decode_k1_multi_mix(const DecodeArgs& a, uint32_t max_frames, hipStream_t st);  // decode_k1_multi_mix.hip
hipError_t launch_decode_k1_multi(const DecodeArgs& a, uint32_t max_frames, hipStream_t st) {
    const hipError_t e = launch_decode_layout<1, LAY_MULTI>(a, max_frames, st);
    return e != hipSuccess ? e : launch_decode_k1_multi_mix(a, max_frames, st);
}
}  // namespace zflac

// decode_k2_stereo.hip -- decode kernel for SampleType container kind 2 (i32), stereo layout.
// One translation unit per (container, layout) so the instantiations compile in parallel.
#define ZFLAC_RING_Q 32  // 128-word rings for 17..32 bits per sample (decode.inc)
#include "decode.inc"

namespace zflac {
hipError_t launch_decode_k2_stereo_mix(const DecodeArgs& a, uint32_t max_frames, hipStream_t st);  // decode_k2_stereo_mix.hip
hipError_t launch_decode_k2_stereo(const DecodeArgs& a, uint32_t max_frames, hipStream_t st) {
    const hipError_t e = launch_decode_layout<2, LAY_STEREO>(a, max_frames, st);
    return e != hipSuccess ? e : launch_decode_k2_stereo_mix(a, max_frames, st);
}
// k_walk for this container: used by the stereo and the 3..8-channel layouts
hipError_t launch_walk_k2(const DecodeArgs& a, uint32_t max_frames, hipStream_t st) {
    return launch_walk_kind<2>(a, max_frames, st);
}
}  // namespace zflac

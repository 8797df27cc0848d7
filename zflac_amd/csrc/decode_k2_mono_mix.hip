// decode_k2_mono_mix.hip -- the MIX decode kernels (waves with CONSTANT / VERBATIM lanes) for
// SampleType container kind 2 (i32), mono layout. Kept out of decode_k2_mono.hip so the
// pure kernels' code object is unchanged by them.
#define ZFLAC_RING_Q 32  // 128-word rings for 17..32 bits per sample (decode.inc)
#include "decode.inc"

namespace zflac {
hipError_t launch_decode_k2_mono_mix(const DecodeArgs& a, uint32_t max_frames, hipStream_t st) {
    return launch_decode_mix<2, LAY_MONO>(a, max_frames, st);
}
}  // namespace zflac

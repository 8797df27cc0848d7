// decode_k0_mono_mix.hip -- the MIX decode kernels (waves with CONSTANT / VERBATIM lanes) for
// SampleType container kind 0 (i8), mono layout. Kept out of decode_k0_mono.hip so the
// pure kernels' code object is unchanged by them.
#include "decode.inc"

namespace zflac {
hipError_t launch_decode_k0_mono_mix(const DecodeArgs& a, uint32_t max_frames, hipStream_t st) {
    return launch_decode_mix<0, LAY_MONO>(a, max_frames, st);
}
}  // namespace zflac

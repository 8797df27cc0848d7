#!/bin/bash
# tools/kmeta.sh <obj.o>...: per-kernel VGPR / SGPR counts and spills of the gfx950 code objects
# in hipcc objects (clang-offload-bundler + llvm-readelf notes). ISA study only.
B=/opt/rocm/lib/llvm/bin
for o in "$@"; do
  t=$(mktemp -d)
  $B/llvm-objcopy --dump-section .hip_fatbin=$t/fat.bin $o 2>/dev/null
  $B/clang-offload-bundler --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=$t/fat.bin --output=$t/dev.o --unbundle 2>/dev/null
  $B/llvm-readelf --notes $t/dev.o 2>/dev/null | python3 -c "
import sys,re
txt=sys.stdin.read()
for blk in txt.split('- .agpr_count')[1:]:
    name=re.search(r'\.name:\s+(\S+)',blk); v=re.search(r'\.vgpr_count:\s+(\d+)',blk); vs=re.search(r'\.vgpr_spill_count:\s+(\d+)',blk)
    ss=re.search(r'\.sgpr_spill_count:\s+(\d+)',blk); pr=re.search(r'\.private_segment_fixed_size:\s+(\d+)',blk)
    if name: print(f'{name.group(1)[:60]:60} vgpr={v.group(1)} vspill={vs.group(1)} sspill={ss.group(1)} scratch={pr.group(1) if pr else \"?\"}')
"
  rm -rf $t
done

#!/bin/bash
# Same-box A/B: walk workgroup size (2 vs 4 waves) x runs in flight (1, 2, 3), twice each.
set -e
mkdir -p gpurun_out/abinf
for i in 1 2; do
for L in zflac_amd/libzflac_hip.so tools/_build/lib_walk256.so; do
for N in 1 2 3; do
  n=$(basename $L .so)
  ZFLAC_HIP_LIB=$L timeout -k 10 200 python bench.py --no-e2e --no-cpu-baseline --no-md5 --no-verify --steps 40 --inflight $N \
    > gpurun_out/abinf/${n}_inf${N}_$i.json 2> gpurun_out/abinf/${n}_inf${N}_$i.err
done; done; done

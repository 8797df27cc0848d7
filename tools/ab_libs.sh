#!/bin/bash
set -e
# Bench A/B of several library builds on one box (ZFLAC_HIP_LIB), alternating, twice.
for i in 1 2; do
for L in tools/_build/libzflac_hip_prev.so tools/_build/lib_x_nocv.so tools/_build/lib_x_nocvalr.so zflac_amd/libzflac_hip.so; do
  n=$(basename $L .so)
  ZFLAC_HIP_LIB=$L timeout -k 10 200 python bench.py --no-e2e --no-cpu-baseline --no-md5 --steps 30 > gpurun_out/ab5_${n}_$i.json 2>gpurun_out/ab5_${n}_$i.err
done; done

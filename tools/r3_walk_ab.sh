#!/bin/bash
# Round-3 A/B: GPU tests, bench with each walk, config rows with both walks.
# Usage: tools/r3_walk_ab.sh <tag>
TAG=${1:-r3c}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-e2e --cpu-seconds 2 > $O/bench_auto.json 2> $O/bench_auto.err || exit $?
ZFLAC_WALK=wave timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-e2e --no-cpu-baseline --no-md5 > $O/bench_wave.json 2> $O/bench_wave.err || exit $?
timeout -k 10 400 python tools/bench_configs.py --walk both --rows "2600 frames,6-channel,32-bit,C3 stereo" --steps 5 --out $O/configs.json > $O/configs.log 2>&1

set -o pipefail
O=gpurun_out/ab3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1 || exit $?
bash tools/ab.sh ab3 2 tools/_build/lib_v29a.so zflac_amd/libzflac_hip.so || exit $?
timeout -k 10 300 python tools/bench_configs.py --rows "C2 mono" --steps 5 --out $O/c2_v30.json > $O/c2_v30.log 2>&1 || exit $?
ZFLAC_HIP_LIB=tools/_build/lib_v30_monostore_abl.so timeout -k 10 300 python tools/bench_configs.py --rows "C2 mono" --steps 5 --out $O/c2_abl.json > $O/c2_abl.log 2>&1

set -o pipefail
T=r6h; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python tools/bench_configs.py --steps 5 --out $O/configs.json > $O/configs.log 2>&1 || { tail -20 $O/configs.log; exit 1; }
ZFLAC_HIP_LIB=tools/_build/lib_A.so timeout -k 10 400 python tools/bench_configs.py --steps 5 --rows "20-bit,32-bit,6-channel,8-bit" --out $O/configs_A.json > $O/configs_A.log 2>&1 || { tail -20 $O/configs_A.log; exit 1; }
python - << 'PY'
import json
for f in ("gpurun_out/r6h/configs.json", "gpurun_out/r6h/configs_A.json"):
    d = json.load(open(f))
    for r in d["rows"]:
        print(f.split("/")[-1][:12], r["row"][:40], r["device_msps"], r["walk_ms"], r["decode_ms"], r["decode_kernel_frac_of_8TBs"], r["bit_exact"])
PY

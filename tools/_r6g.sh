set -o pipefail
T=r6g
bash tools/gpu.sh check $T || { tail -30 gpurun_out/$T/gputest.txt; exit 1; }
tail -2 gpurun_out/$T/gputest.txt; cat gpurun_out/$T/smoke.txt | tail -2
python -c "import json;d=json.loads(open('gpurun_out/$T/bench.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline'], d.get('device_md5',{}).get('decode_plus_md5_msps_rank0'))"
bash tools/gpu.sh pmc $T || { tail -20 gpurun_out/$T/pmc_summary.log; exit 1; }
tail -5 gpurun_out/$T/pmc_summary.log
bash tools/gpu.sh profile $T || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/$T/bench20.json 2> gpurun_out/$T/bench20.err || exit 1
python -c "import json;d=json.loads(open('gpurun_out/$T/bench20.json').read().strip().splitlines()[-1]);print('20 steps', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'])"

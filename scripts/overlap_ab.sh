set -e
for m in off after before off after before; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 --warmup 5 --overlap $m > gpurun_out/ov_$m.json 2>gpurun_out/ov_err.log
  python -c "import json,sys; d=json.loads(open('gpurun_out/ov_$m.json').read().strip().splitlines()[-1]); print('$m', round(d['ms_per_step'],4), d['roofline']['achieved'])"
done

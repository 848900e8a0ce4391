#!/bin/bash
# Round 6 re-entry, final library: the serial step (the bench default) and the
# overlapped step (--overlap on: the codebook walk on a side stream beside
# BatchNorm + assign), three interleaved rounds of 40 steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06y9
mkdir -p $O
for r in 1 2 3; do
  for ov in off on; do
    timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --overlap $ov > $O/ov_${ov}_$r.json 2> $O/ov_${ov}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/ov_${ov}_$r.json').read().strip().splitlines()[-1]); print('$r overlap $ov', 'ms/step %.4f' % d['ms_per_step'], 'assign us %.1f' % (d['kernels']['vq_assign']['ms_per_launch'] * 1e3), d['config']['schedule'])"
  done
done

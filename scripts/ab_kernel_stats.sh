#!/bin/bash
# Per-kernel rocprofv3 statistics of the bench step for library variants
# (VQGNN_LIB), interleaved twice:  ab_kernel_stats.sh "default name ..." [regex]
# ("default" = the in-tree library; name = vq-gnn_amd/lib/ab_<name>.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-abks}
mkdir -p $O
PAT="${2:-.}"
for rep in 1 2; do
  for n in $1; do
    if [ "$n" = "default" ]; then unset VQGNN_LIB; else export VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_$n.so; fi
    d=$O/${n}_$rep
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv \
      -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $d.log 2>&1 || exit 1
    python3 - "$d/run_kernel_stats.csv" "$n $rep" "$PAT" <<'PY'
import csv, re, sys
for x in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[3], x["Name"]):
        print(sys.argv[2], x["Name"][:44], x["Calls"], "%.2f us" % (float(x["AverageNs"]) / 1e3))
PY
  done
done

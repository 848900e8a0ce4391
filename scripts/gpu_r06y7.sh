#!/bin/bash
# Round 6 re-entry: what the fused assign's final slab fold costs -- the
# probe build without it (ab_noflush, -DVQGNN_ASG_NO_FLUSH=1, results
# invalid) against the shipped library, scripts/assign_probe.py (static
# codebook, arxiv shapes, M = 256 and 1,024), three interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
L=$PWD/vq-gnn_amd/lib
for rep in 1 2 3; do
  for m in 256 1024; do
    for lib in libvqgnn ab_noflush; do
      echo "== rep $rep M=$m $lib"
      M=$m VQGNN_LIB=$L/$lib.so timeout -k 10 120 python scripts/assign_probe.py || exit 1
    done
  done
done

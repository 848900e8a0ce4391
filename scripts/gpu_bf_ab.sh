#!/bin/bash
# Branch-free codebook-source loads against the default library (probe
# parity and timing, bench A/B): ab_bf (codebook edges' X gathers past the
# buffer range) or ab_bf2 (codebook edges gather X row 0), both built by
# scripts/build_variant.sh from copies of spmm_tasks.hip
bash "$(dirname "$0")/gpu_lib_ab.sh" "${1:-bf2}"

#!/bin/bash
# Build a library variant with one source file replaced (A/B measurements):
#   build_variant.sh <name> <replaced.hip> <replacement file>
# -> vq-gnn_amd/lib/ab_<name>.so (travels to the GPU box; select it with
#    VQGNN_LIB=vq-gnn_amd/lib/ab_<name>.so).  The replaced file is compiled
#    with -DVQGNN_EXPERIMENTS: its measurement knobs (VQGNN_TASK_U/G,
#    VQGNN_ASG_*, VQGNN_ASSIGN_MSWEEP, VQGNN_TASK_DBG, ...) read the
#    environment there and only there -- the default library ignores them.
#    EXTRA_FLAGS: more hipcc flags for the replaced file.  EXP_ALSO: more
#    in-tree sources (space separated) compiled with -DVQGNN_EXPERIMENTS too.
set -e
cd "$(dirname "$0")/../vq-gnn_amd/csrc"
name=$1; src=$2; repl=$3
make -s -j8 >/dev/null
tmp=../lib/obj/ab_$name
mkdir -p $tmp
cp "$repl" $tmp/$src
objs=""
for f in $(sed -n 's/^SRCS := //p;s/^         //p' Makefile | tr ' ' '\n' | grep hip); do
  if [ "$f" = "$src" ]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++20 -ffp-contract=off -Wall \
      -Wno-unused-function -munsafe-fp-atomics -DVQGNN_EXPERIMENTS $EXTRA_FLAGS -I$PWD -c $tmp/$src -o $tmp/${src%.hip}.o
    objs="$objs $tmp/${src%.hip}.o"
  elif [[ " $EXP_ALSO " == *" $f "* ]]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++20 -ffp-contract=off -Wall \
      -Wno-unused-function -munsafe-fp-atomics -DVQGNN_EXPERIMENTS $(test $f = vq_kernels.hip && echo -fno-slp-vectorize) \
      -I$PWD -c $f -o $tmp/${f%.hip}.o
    objs="$objs $tmp/${f%.hip}.o"
  else
    objs="$objs ../lib/obj/${f%.hip}.o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/ab_$name.so $objs
echo "built vq-gnn_amd/lib/ab_$name.so"

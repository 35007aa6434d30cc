#!/bin/bash
# Instrumented variants of the library for profiling experiments: agg_bucket_fast_tiled.hip built
# with -D<flag>, linked with the other objects of the in-tree build into tiflash_amd/exp/lib_<flag>.so
# (select one with TFA_LIB_PATH).  Usage: tools/build_exp.sh FLAG[,FLAG2] ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/tiflash_amd/csrc
mkdir -p $ROOT/tiflash_amd/exp /tmp/tfg_exp
for spec in "$@"; do
  defs=""
  for f in ${spec//,/ }; do defs="$defs -D$f"; done
  name=$(echo $spec | tr ',' '_')
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $defs -c $CS/agg_bucket_fast_tiled.hip -o /tmp/tfg_exp/$name.o &
done
wait
for spec in "$@"; do
  name=$(echo $spec | tr ',' '_')
  objs=$(ls $CS/build/*.o | grep -v agg_bucket_fast_tiled.o)
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $ROOT/tiflash_amd/exp/lib_$name.so $objs /tmp/tfg_exp/$name.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo built $ROOT/tiflash_amd/exp/lib_$name.so
done

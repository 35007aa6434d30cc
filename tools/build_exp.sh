#!/bin/bash
# Instrumented variants of the library for profiling experiments: the sources in $EXP_SRCS
# (default agg_bucket_fast_tiled.hip) built with -D<flag>, linked with the other objects of the
# in-tree build into tiflash_amd/exp/lib_<flag>.so (select one with TFA_LIB_PATH).
# Usage: [EXP_SRCS="agg.hip agg_bucket_fast_tiled.hip"] tools/build_exp.sh FLAG[,FLAG2] ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/tiflash_amd/csrc
SRCS=${EXP_SRCS:-agg_bucket_fast_tiled.hip}
mkdir -p $ROOT/tiflash_amd/exp /tmp/tfg_exp
for spec in "$@"; do
  defs=""
  for f in ${spec//,/ }; do defs="$defs -D$f"; done
  name=$(echo $spec | tr ',' '_')
  for s in $SRCS; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $defs -c $CS/$s -o /tmp/tfg_exp/${name}__${s%.hip}.o &
  done
done
wait
for spec in "$@"; do
  name=$(echo $spec | tr ',' '_')
  objs=""
  for o in $CS/build/*.o; do
    b=$(basename $o .o)
    skip=0
    for s in $SRCS; do [ "$b" = "${s%.hip}" ] && skip=1; done
    [ $skip = 0 ] && objs="$objs $o"
  done
  for s in $SRCS; do objs="$objs /tmp/tfg_exp/${name}__${s%.hip}.o"; done
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $ROOT/tiflash_amd/exp/lib_$name.so $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo built $ROOT/tiflash_amd/exp/lib_$name.so
done

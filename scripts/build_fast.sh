#!/bin/bash
# Dev: quick variant library for config-3 experiments: compiles only the host side and
# capacity class A (NMPC_TU_CLASS=1) from $2 and links the other classes' objects from a
# cache built once from $3 (default: the checked-out source).  usage: build_fast.sh out.so src.hip [cache_src]
OUT=$1; SRC=$2; CSRC=${3:-/root/repo/mpc-implementation_amd/csrc/nmpc_solve.hip}
C=/tmp/basecache
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -disable-machine-licm -Wno-unused-result -Wno-unused-value -I /root/repo/include"
pids=""
for tu in 2 3 4 5 6 7; do
  [ -f $C/$tu.o ] || { /opt/rocm/bin/hipcc $F -DNMPC_TU_CLASS=$tu -c $CSRC -o $C/$tu.o & pids="$pids $!"; }
done
T=$(mktemp -d)
/opt/rocm/bin/hipcc $F -DNMPC_TU_HOST -c $SRC -o $T/h.o & pids="$pids $!"
/opt/rocm/bin/hipcc $F -DNMPC_TU_CLASS=1 -c $SRC -o $T/1.o & pids="$pids $!"
for p in $pids; do wait $p || exit 1; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared $T/h.o $T/1.o $C/2.o $C/3.o $C/4.o $C/5.o $C/6.o $C/7.o -o $OUT && rm -rf $T && echo built $OUT

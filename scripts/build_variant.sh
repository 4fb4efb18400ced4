#!/bin/bash
# build a variant library: $1 = output .so, rest = extra flags (flag "NOLICM" drops -disable-machine-licm)
OUT=$1; shift
LICM="-mllvm -disable-machine-licm"
EXTRA=""
for a in "$@"; do if [ "$a" == "NOLICM" ]; then LICM=""; else EXTRA="$EXTRA $a"; fi; done
SRC=${NMPC_SRC:-/root/repo/mpc-implementation_amd/csrc/nmpc_solve.hip}
T=$(mktemp -d)
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC $LICM -Wno-unused-result -Wno-unused-value $EXTRA -I /root/repo/include"
pids=""
for tu in HOST 1 2 3 4 5 6 7; do
  if [ $tu == HOST ]; then D=-DNMPC_TU_HOST; else D=-DNMPC_TU_CLASS=$tu; fi
  /opt/rocm/bin/hipcc $F $D -c $SRC -o $T/$tu.o & pids="$pids $!"
done
for p in $pids; do wait $p || exit 1; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared $T/*.o -o $OUT && rm -rf $T && echo built $OUT

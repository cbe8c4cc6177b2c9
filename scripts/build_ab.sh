#!/bin/bash
# A/B builds of one translation unit with extra flags, linked against the other objects
# of the current build: ab/libgpmpc_NAME.so (load it with GPMPC_LIB=...).
#   bash scripts/build_ab.sh NAME SRC.hip "-DFLAG=1 ..."
set -euo pipefail
NAME=$1; SRC=$2; XF=${3:-}
C=gp_mpc_rocket_landing_amd/csrc
mkdir -p ab
make -s -C $C >/dev/null
OBJ=$(basename "$SRC" .hip)
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC $XF -c $C/$SRC -o /tmp/ab_${NAME}_$OBJ.o
OTHERS=$(ls $C/build/*.o | grep -v "/$OBJ.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OTHERS /tmp/ab_${NAME}_$OBJ.o -ldl -o ab/libgpmpc_$NAME.so
echo "ab/libgpmpc_$NAME.so"

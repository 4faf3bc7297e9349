#!/bin/bash
# Builds an A/B variant of the library that differs only in env_step.hip:
#   scripts/build_env_variant.sh NAME "EXTRA HIPCC FLAGS" [GIT_REV]
# -> dgppo_fov_amd/lib/libdgppo_hip_NAME.so (env_step.hip from GIT_REV if given, else the working tree; every other
# object is the in-tree build).  Run `make` first.  Used by scripts/ab_env_multi.sh.
set -e
cd "$(dirname "$0")/.."
NAME=$1; FLAGS=$2; REV=$3
OBJ=dgppo_fov_amd/_build
SRC=dgppo_fov_amd/csrc/env_step.hip
if [ -n "$REV" ]; then
  mkdir -p $OBJ/rev_$NAME
  git show "$REV:$SRC" > $OBJ/rev_$NAME/env_step.hip
  SRC=$OBJ/rev_$NAME/env_step.hip
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Iinclude -Idgppo_fov_amd/csrc $FLAGS \
  -c $SRC -o $OBJ/env_step_$NAME.o
OBJS=$(ls $OBJ/*.o | grep -v "env_step" | tr '\n' ' ')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o dgppo_fov_amd/lib/libdgppo_hip_$NAME.so $OBJS $OBJ/env_step_$NAME.o
echo "built dgppo_fov_amd/lib/libdgppo_hip_$NAME.so"

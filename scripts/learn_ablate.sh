#!/bin/bash
# Identical-seed learning ablations of the DGPPO collapse (VERDICT r02 "Next" #1), 300 updates each through
# train.py / test.py (scripts/learning_run.py; per-update train/reward, train/unsafe_frac, train/act_drift,
# safe_data, Vh loss, clip_frac, entropy in update_curve).  Usage: scripts/learn_ablate.sh [group]
#   group lt  : LidarTarget n=2 obs=0 --rnn-step 128 (where InforMARL learns)
#   group mp  : MPETarget n=2 obs=0 --batch-size 4096 (4 minibatches per update)
#   group ent : the entropy-term ablations (--coef-ent 0) at the reference default rnn_step 16
# Results: gpurun_out/abl_<name>/learning_run.json.  Stops at the first failing run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
group=${1:-lt}
STEPS=${STEPS:-300}
run() {  # name, env vars..., -- , learning_run args...
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 600 python -u scripts/learning_run.py --out gpurun_out/abl_$name --steps $STEPS \
    --eval-interval 50 --epi 32 "$@" > gpurun_out/abl_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
FS=DGPPO_DEBUG_FORCE_SAFE=1
LT=(--env LidarTarget -n 2 --obs 0 --rnn-step 128)
MP=(--env MPETarget -n 2 --obs 0 --batch-size 4096)
case $group in
  lt)
    run lt_inf X=0 -- "${LT[@]}" --algo informarl
    run lt_dg_c0_fs $FS -- "${LT[@]}" --algo dgppo --cbf-weight 0
    run lt_dg_c0_fs_s0 $FS DGPPO_STREAMS=0 -- "${LT[@]}" --algo dgppo --cbf-weight 0
    run lt_dg_c0 X=0 -- "${LT[@]}" --algo dgppo --cbf-weight 0
    run lt_dg X=0 -- "${LT[@]}" --algo dgppo
    ;;
  mp)
    run mp_inf X=0 -- "${MP[@]}" --algo informarl
    run mp_dg_c0_fs $FS -- "${MP[@]}" --algo dgppo --cbf-weight 0
    run mp_dg_c0 X=0 -- "${MP[@]}" --algo dgppo --cbf-weight 0
    run mp_dg X=0 -- "${MP[@]}" --algo dgppo
    ;;
  ent)
    run lt16_inf_ent0 X=0 -- --env LidarTarget -n 2 --obs 0 --algo informarl --coef-ent 0
    run lt_dg_ent0 X=0 -- "${LT[@]}" --algo dgppo --coef-ent 0
    run mp_dg_ent0 X=0 -- "${MP[@]}" --algo dgppo --coef-ent 0
    ;;
  seeds)
    for sd in 1 2 3; do run lt_dg_seed$sd X=0 -- "${LT[@]}" --algo dgppo --seed $sd; done
    ;;
  quickstart)  # the reference README's quickstart: python train.py --env LidarSpread --algo dgppo -n 3 --obs 3
    for sd in 0 1; do STEPS=2000 run qs_dg_seed$sd X=0 -- --env LidarSpread -n 3 --obs 3 --algo dgppo --seed $sd; done
    ;;
esac

#!/bin/bash
# Long learning runs of the README quickstart (LidarSpread n=3 obs=3, reference defaults: 128 envs,
# batch 16384, --steps 200000 schedule, eval every 50 updates on 32 envs) spanning several gpurun calls.
# Each call resumes every run found under runs_long/ (copied back from gpurun_out/long/ by the caller
# between calls: scripts/long_sync.sh), trains for MIN minutes, saves a resumable state and prunes old
# checkpoints.  Runs go side by side on the one GPU (each is launch-bound at 128 envs).
#   RUNS="dgppo:0 informarl:0" MIN=17 bash scripts/long_run.sh
# ENV (default LidarSpread) picks the env of the quickstart command (-n 3 --obs 3), e.g. ENV=MPESpread.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/long
MIN=${MIN:-17}
ENV=${ENV:-LidarSpread}
pids=()
for spec in ${RUNS:-dgppo:0 informarl:0}; do
  algo=${spec%%:*}; seed=${spec##*:}
  base=gpurun_out/long/$ENV/$algo
  mkdir -p $base
  prev=$(ls -d runs_long/$ENV/$algo/seed${seed}_* 2>/dev/null | head -1)
  args=(--env $ENV -n 3 --obs 3 --algo $algo --seed $seed --steps 200000 --eval-interval 50
        --save-interval 100000 --log-interval 50 --max-minutes $MIN --log-dir gpurun_out/long)
  if [ -n "$prev" ]; then
    cp -r "$prev" $base/
    args+=(--resume $base/$(basename "$prev"))
  fi
  timeout -k 10 $(( MIN * 60 + 150 )) python -u train.py "${args[@]}" > gpurun_out/long/${ENV}_${algo}_seed${seed}.log 2>&1 &
  pids+=($!)
done
rc=0
while true; do  # progress for gpurun's liveness check
  sleep 60; alive=0
  for p in "${pids[@]}"; do kill -0 $p 2>/dev/null && alive=1; done
  for f in gpurun_out/long/*.log; do echo "$f: $(grep '^step' $f | tail -1)"; done
  [ $alive = 0 ] && break
done
for p in "${pids[@]}"; do wait $p || rc=$?; done
# keep only the newest checkpoint of each run (plus step 0) so the merge stays small
for m in gpurun_out/long/$ENV/*/seed*/models; do
  keep=$(ls $m | sort -n | tail -1)
  for d in $(ls $m); do [ "$d" = "$keep" ] || [ "$d" = "0" ] || rm -rf "$m/$d"; done
done
tail -3 gpurun_out/long/*.log
exit $rc

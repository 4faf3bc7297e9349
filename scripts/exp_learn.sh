set -e
run() { tag=$1; shift; timeout -k 10 500 python -u scripts/learning_run.py --epi 64 --out gpurun_out/x_$tag "$@" > gpurun_out/x_$tag.log 2>&1; python -c "
import json; d=json.load(open('gpurun_out/x_$tag/learning_run.json'))
print('$tag eval', [(r['step'], round(r['eval/reward'],3), round(r['eval/unsafe_frac'],2)) for r in d['eval_curve']])
print('$tag train', d['train_curve'][::2])"; }
run inf_r128 --algo informarl --env LidarTarget -n 2 --obs 0 --steps 300 --eval-interval 50 --rnn-step 128
run dg_r128 --algo dgppo --steps 600 --eval-interval 100 --rnn-step 128

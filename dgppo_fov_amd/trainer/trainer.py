"""Trainer (dgppo/trainer/trainer.py:17-140): collect -> update loop with periodic deterministic
evaluation and checkpoints.  Same constructor and `params` contract as the reference; logging goes
to `<log_dir>/log.jsonl` (+ stdout) instead of wandb (not installed, no network).  Multi-GPU: every
rank trains on its own env shard (`DGPPO` all-reduces the gradients); rank 0 evaluates, logs and
saves."""
from __future__ import annotations

import json
import os
from time import time

import numpy as np
import torch.distributed as dist

from ..algo.dgppo import DGPPO
from ..env.base import MultiAgentEnv
from ..trainer.rollout import RolloutEngine
from .utils import eval_info


class Trainer:
    def __init__(self, env: MultiAgentEnv, env_test: MultiAgentEnv, algo: DGPPO, gamma: float, n_env_train: int,
                 n_env_test: int, log_dir: str, seed: int, params: dict, save_log: bool = True):
        self.env, self.env_test, self.algo = env, env_test, algo
        self.gamma, self.n_env_train, self.n_env_test = gamma, n_env_train, n_env_test
        self.log_dir, self.seed = log_dir, seed
        if Trainer._check_params(params):
            self.params = params
        self.rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        self.save_log = save_log and self.rank == 0
        if self.save_log:
            os.makedirs(log_dir, exist_ok=True)
            self.model_dir = os.path.join(log_dir, "models")
            os.makedirs(self.model_dir, exist_ok=True)
        self.steps = params["training_steps"]
        self.eval_interval = params["eval_interval"]
        self.eval_epi = params["eval_epi"]
        self.save_interval = params["save_interval"]
        self.update_steps = 0
        self.start_step = 0
        self.rng = np.random.default_rng(seed)
        self._test_engine = None
        # not in the reference (it logs every update to wandb and trains in one process lifetime):
        # log.jsonl keeps every log_interval-th update, and train() returns after max_minutes of wall
        # time with a resumable state (save_state / load_state), so a long run can span processes
        self.log_interval = int(params.get("log_interval", 1))
        self.max_minutes = params.get("max_minutes")

    @staticmethod
    def _check_params(params: dict) -> bool:
        assert "run_name" in params, "run_name not found in params"
        assert "training_steps" in params, "training_steps not found in params"
        assert "eval_interval" in params, "eval_interval not found in params"
        assert params["eval_interval"] > 0, "eval_interval must be positive"
        assert "eval_epi" in params, "eval_epi not found in params"
        assert params["eval_epi"] >= 1, "eval_epi must be greater than or equal to 1"
        assert "save_interval" in params, "save_interval not found in params"
        assert params["save_interval"] > 0, "save_interval must be positive"
        return True

    def _log(self, record: dict):
        if self.save_log:
            with open(os.path.join(self.log_dir, "log.jsonl"), "a") as f:
                f.write(json.dumps(record) + "\n")

    def evaluate(self, key: int) -> dict:
        """test_rollout with the deterministic policy on n_env_test envs (trainer.py:85-116)."""
        assert self.n_env_test <= 1_000, "n_env_test must be less than or equal to 1_000"
        if self._test_engine is None:
            self._test_engine = RolloutEngine(self.env_test, self.n_env_test, self.env_test.max_episode_steps,
                                              self.algo.device, actor=self.algo.actor, mode=RolloutEngine.MODE_DET)
        r = self._test_engine.run(key)
        return eval_info(r.rewards, r.costs)

    # ---- resumable state (params + optimiser + RNG; the reference saves params only) ----------
    STATE_FILE = "trainer_state.json"

    def save_state(self, next_step: int):
        """models/<next_step>/ (params + Adam moments + counters, algo.save) and trainer_state.json: the next
        step and every host RNG the loop draws from, so load_state() continues the exact sequence.  The model
        directory keeps the periodic saves' meaning, models/<k> = the state BEFORE update k (so a stop never
        overwrites an earlier save with other parameters, and models/0 stays the initial parameters)."""
        if not self.save_log:
            return
        self.algo.save(self.model_dir, next_step)
        st = {"next_step": next_step, "update_steps": self.update_steps, "model_step": next_step,
              "trainer_rng": self.rng.bit_generator.state, "algo_key": self.algo.key.bit_generator.state,
              "algo_np_rng": self.algo.np_rng.bit_generator.state}
        tmp = os.path.join(self.log_dir, self.STATE_FILE + ".tmp")
        with open(tmp, "w") as f:
            json.dump(st, f)
        os.replace(tmp, os.path.join(self.log_dir, self.STATE_FILE))

    def load_state(self, run_dir: str):
        """Continue a run saved by save_state (its log_dir): parameters, Adam state, step and RNG streams."""
        with open(os.path.join(run_dir, self.STATE_FILE)) as f:
            st = json.load(f)
        self.algo.load(os.path.join(run_dir, "models"), st["model_step"])
        self.rng.bit_generator.state = st["trainer_rng"]
        self.algo.key.bit_generator.state = st["algo_key"]
        self.algo.np_rng.bit_generator.state = st["algo_np_rng"]
        self.start_step, self.update_steps = st["next_step"], st["update_steps"]
        return st

    def _out_of_time(self, start_time: float) -> bool:
        """The --max-minutes stop decision, taken by rank 0 and broadcast, so every rank stops at the same step
        (a rank that stopped on its own clock would leave the others blocked in the gradient all-reduce)."""
        if self.max_minutes is None:
            return False
        stop = time() - start_time > 60.0 * float(self.max_minutes)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            flag = [bool(stop)]
            dist.broadcast_object_list(flag, src=0)
            stop = bool(flag[0])
        return stop

    def train(self):
        start_time = time()
        test_key = int(self.seed)
        for step in range(self.start_step, self.steps + 1):
            if self._out_of_time(start_time):
                self.save_state(step)
                print(f"> stopping after {time() - start_time:.0f}s at step {step} (resume with --resume)", flush=True)
                return False
            if step % self.eval_interval == 0 and self.rank == 0:
                info = self.evaluate(test_key)
                print(f"step: {step:3}, time: {time() - start_time:5.0f}s, reward: {info['eval/reward']:9.4f}, "
                      f"min/max reward: {info['eval/reward_min']:7.2f}/{info['eval/reward_max']:7.2f}, "
                      f"cost: {info['eval/cost']:8.4f}, unsafe_frac: {info['eval/unsafe_frac']:6.2f}", flush=True)
                self._log({"step": self.update_steps, **info})
            if self.save_log and step % self.save_interval == 0:
                self.algo.save(self.model_dir, step)
            key = int(self.rng.integers(0, 2 ** 62))
            rollouts = self.algo.collect(self.algo.params, key, n_env=self.n_env_train)
            train_stats = self._train_stats(rollouts)  # device scalars: no host sync before the update
            update_info = self.algo.update(rollouts, step)
            if step % self.log_interval == 0:
                self._log({"step": self.update_steps, **update_info, **self._read_stats(train_stats)})
            self.update_steps += 1
        if self.max_minutes is not None:
            self.save_state(self.steps + 1)
        return True

    def _train_stats(self, rollouts):
        """The stochastic rollouts' own metrics as ONE device vector, enqueued right after collect (the next
        collect overwrites the rollout buffers): [episode return, unsafe_frac (eval_info's definitions),
        mean |E_(env,t)[action]| over (agent, dim) -- a policy-mean drift indicator]."""
        import torch

        r, c, a = rollouts.rewards, rollouts.costs, rollouts.actions
        return torch.stack([r.sum(-1).mean(), (c.amax(-1).amax(-2) >= 1e-6).float().mean(),
                            a.mean((0, 1)).abs().mean()])

    def _read_stats(self, v) -> dict:
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(v)
            v = v / dist.get_world_size()
        s = v.tolist()
        return {"train/reward": s[0], "train/unsafe_frac": s[1], "train/act_drift": s[2]}

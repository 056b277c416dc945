"""GPU-resident deep-sets DQN.

Restates envs/dqn_deepset.py:44-231 on device tensors: epsilon-greedy with ONE
random.random() deciding exploration for all envs (:127), masked argmax of Q (:134-142),
an SB3-style replay buffer resident in HBM (buffer_size // num_envs slots of num_envs
transitions, uniform (slot, env) sampling; next_obs stored as returned — the reset obs
for finished envs, as the reference stores it, :158-174), TD target from the target
network's max (:180-186), MSE loss, Adam, hard target copy every
target_network_frequency steps (tau = 1, :199-203).  total_timesteps counts VECTOR steps
(:122).

On a GPU the decisions the reference makes on the host are drawn by kernels (device RNG):
the per-step explore draw random.random() < epsilon (:127) by lb_dqn_act, the replay
sample (:177) by lb_replay_sample (Philox keyed by the learner seed and the vector step: the
same distributions as the reference's generators, not their streams).  A train period --
train_frequency vector steps and the train step -- then holds no host decision and replays
as ONE HIP graph (period_graph=True, the default with train_graph); the eager run of the
same kernels trains identically (tests/test_gpu_learners.py).

Multi-GPU: gradients averaged with one all_reduce per train step (RCCL); every rank keeps
its own envs and replay; the logged episode return is the mean over every rank's finished
episodes (one 2-double all_reduce per log line).
"""
import os
import random
import time
from copy import deepcopy

import numpy as np
import torch
import torch.nn.functional as F
from torch import optim

from . import _native, fused, fused_train
from . import dist as lbdist
from .deepsets import DQNDeepSetAgent, HUGE_NEG, allreduce_gradients


DQN_STEPS_MAX = 32  # lb_dqn_steps' longest launch (include/lbk8s.h)


def linear_schedule(start_e: float, end_e: float, duration: float, t: int) -> float:
    slope = (end_e - start_e) / duration
    return max(slope * t + start_e, end_e)


class DeviceReplayBuffer:
    """SB3 ReplayBuffer semantics (n_envs-major circular storage) with device tensors.

    The write position also lives on the device (`pos_t`), so `add_device` is
    graph-capturable: one captured vector step serves every slot.  The host mirrors it
    (`pos`, `full`) for the sampling bound."""

    def __init__(self, buffer_size, num_envs, obs_shape, device, generator):
        self.n_envs = num_envs
        self.size = max(buffer_size // num_envs, 1)
        self.obs = torch.zeros((self.size, num_envs) + tuple(obs_shape), device=device)
        self.next_obs = torch.zeros_like(self.obs)
        self.actions = torch.zeros((self.size, num_envs), dtype=torch.long, device=device)
        self.rewards = torch.zeros((self.size, num_envs), device=device)
        self.dones = torch.zeros((self.size, num_envs), device=device)
        self.pos, self.full = 0, False
        self.pos_t = torch.zeros(1, dtype=torch.long, device=device)
        # lb_replay_add's slot words: the launch reads pp[parity], writes pp[1 - parity]
        self.pos_pp = torch.zeros(2, dtype=torch.long, device=device)
        self.gen = generator

    def add_device(self, obs, next_obs, actions, rewards, dones):
        """Device part of add(): write slot pos_t, advance pos_t (no host sync)."""
        i = self.pos_t
        self.obs.index_copy_(0, i, obs[None])
        self.next_obs.index_copy_(0, i, next_obs[None])
        self.actions.index_copy_(0, i, actions.to(torch.long)[None])
        self.rewards.index_copy_(0, i, rewards[None])
        self.dones.index_copy_(0, i, dones[None])
        self.pos_t.add_(1).remainder_(self.size)

    def add_fused(self, obs, next_obs, actions_i32, rewards, done_u8, ep_stats, ep_sum, ep_cnt, parity):
        """add_device + obs <- next_obs + per-env finished-episode sums as ONE launch
        (lb_replay_add); the device slot lives in pos_pp[parity] and moves to the other word."""
        B = self.n_envs
        pp = self.pos_pp.data_ptr()
        _native.check(_native.lib().lb_replay_add(
            B, int(obs[0].numel()), self.size, pp + 8 * parity, pp + 8 * (1 - parity), obs.data_ptr(),
            next_obs.data_ptr(), actions_i32.data_ptr(), rewards.data_ptr(), done_u8.data_ptr(),
            ep_stats.data_ptr(), self.obs.data_ptr(), self.next_obs.data_ptr(), self.actions.data_ptr(),
            self.rewards.data_ptr(), self.dones.data_ptr(), ep_sum.data_ptr(), ep_cnt.data_ptr(),
            torch.cuda.current_stream(obs.device).cuda_stream))

    def advance_host(self):
        self.pos += 1
        if self.pos == self.size:
            self.full, self.pos = True, 0

    def add(self, obs, next_obs, actions, rewards, dones):
        self.add_device(obs, next_obs, actions, rewards, dones)
        self.advance_host()

    def clear(self):
        self.pos, self.full = 0, False
        self.pos_t.zero_()
        self.pos_pp.zero_()

    def _indices(self, batch_size):
        upper = self.size if self.full else self.pos
        dev = self.obs.device
        bi = torch.randint(0, upper, (batch_size,), device=dev, generator=self.gen)
        ei = torch.randint(0, self.n_envs, (batch_size,), device=dev, generator=self.gen)
        return bi, ei

    def sample(self, batch_size):
        bi, ei = self._indices(batch_size)
        return (self.obs[bi, ei], self.actions[bi, ei][:, None], self.next_obs[bi, ei],
                self.dones[bi, ei][:, None], self.rewards[bi, ei][:, None])

    def sample_into(self, batch_size, out):
        """sample() (the same draws, the same values) into the fixed buffers `out` = (obs,
        actions, next_obs, dones, rewards) of a captured train step."""
        bi, ei = self._indices(batch_size)
        flat = bi * self.n_envs + ei
        for src, dst in zip((self.obs, self.actions, self.next_obs, self.dones, self.rewards), out):
            torch.index_select(src.reshape((-1,) + tuple(src.shape[2:])), 0, flat,
                               out=dst.view((batch_size,) + tuple(src.shape[2:])))


def dqn_loss(q_network, target_network, obs, actions, next_obs, rewards, dones, gamma):
    """dqn_deepset.py:180-187 -> (loss, td_target, old_val).  With the fused kernels (a HIP
    device) the TD target, the squared errors and the loss's gradient are one launch
    (fused_train.dqn_head)."""
    if fused.ENABLED and obs.is_cuda and fused_train.supported(q_network.q_network.net, obs):
        if (obs.shape[1] <= fused_train.PAIR_MAX_ELEMENTS and next_obs.shape == obs.shape and torch.is_grad_enabled()
                and fused._geometry_ok(target_network.q_network.net, next_obs)):
            # (the target's Q(next_obs) and the trained forward in one launch)
            q, q_next = fused_train.q_train_with_target(q_network, q_network.q_network.net, obs, target_network,
                                                        next_obs)
            return fused_train.dqn_head(q, q_next, actions, rewards, dones, gamma)
        with torch.no_grad():
            q_next = fused.q_forward(target_network, next_obs)
        return fused_train.dqn_head(q_network(obs), q_next, actions, rewards, dones, gamma)
    with torch.no_grad():
        target_max, _ = fused.q_forward(target_network, next_obs).max(dim=1)
        td_target = rewards.flatten() + gamma * target_max * (1 - dones.flatten())
    old_val = q_network(obs).gather(1, actions).squeeze()
    return F.mse_loss(td_target, old_val), td_target, old_val


class DQN_DeepSets:
    def __init__(self, env, seed=1, torch_deterministic=True, num_steps: int = 100, learning_rate=2.5e-4,
                 buffer_size=10000, gamma=0.99, tau=1.0, n_minibatches: int = 4, target_network_frequency=500,
                 batch_size=128, start_e=1, end_e=0.05, exploration_fraction=0.5, learning_starts=10000,
                 train_frequency=10, device=None, log_fn=None, num_envs=None, tensorboard_log=None,
                 train_graph=None, period_graph=None, device_rng=None, multi_step=None):
        # num_envs / tensorboard_log: accepted for signature compatibility with
        # dqn_deepset.py:46-67 (the env's num_envs is used; there is no tensorboard writer)
        self.env = env
        self.device = torch.device(device) if device is not None else env.device
        self.num_envs = env.num_envs
        self.num_steps, self.seed, self.learning_rate = num_steps, seed, learning_rate
        self.buffer_size, self.gamma, self.tau = buffer_size, gamma, tau
        self.target_network_frequency, self.batch_size = target_network_frequency, batch_size
        self.start_e, self.end_e, self.exploration_fraction = start_e, end_e, exploration_fraction
        self.learning_starts, self.train_frequency = learning_starts, train_frequency
        self.log_fn = log_fn or (lambda d: None)
        random.seed(seed)
        np.random.seed(seed)
        torch.manual_seed(seed)
        if torch_deterministic:
            torch.backends.cudnn.deterministic = True
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)
        self.q_network = DQNDeepSetAgent(env).to(self.device)
        if lbdist.is_multi():
            lbdist.broadcast_parameters(self.q_network)  # replicas start from rank 0's weights
        self.target_network = deepcopy(self.q_network)
        # the train step (loss, backward, Adam) as a HIP graph replayed on fixed sample
        # buffers: ~60 launches per train step otherwise, the host-bound part of config 5
        self.train_graph = (self.device.type == "cuda") if train_graph is None else bool(train_graph)
        # on a HIP device, torch's fused Adam: one multi-tensor kernel per train step
        self.optimizer = optim.Adam(self.q_network.parameters(), lr=learning_rate,
                                    fused=(self.device.type == "cuda" and os.environ.get("LBK8S_FUSED_ADAM", "1") == "1")
                                    or None, capturable=self.train_graph)
        self._multi = lbdist.is_multi()
        self._gflat = torch.zeros(sum(p.numel() for p in self.q_network.parameters()), device=self.device) \
            if self._multi else None
        self._tgraphs = None
        self.rb = DeviceReplayBuffer(buffer_size, self.num_envs, env.observation_space.shape, self.device, self.gen)
        self._act = torch.zeros(self.num_envs, dtype=torch.int32, device=self.device)
        self._done_u8 = torch.zeros(self.num_envs, dtype=torch.uint8, device=self.device)
        self._rew = torch.zeros(self.num_envs, device=self.device)
        self._next_obs = torch.zeros((self.num_envs,) + tuple(env.observation_space.shape), device=self.device)
        self.episode_returns = []
        # per-env finished-episode sums (reduced when flushed)
        self._ep_sum = torch.zeros(self.num_envs, dtype=torch.float64, device=self.device)
        self._ep_cnt = torch.zeros(self.num_envs, dtype=torch.float64, device=self.device)
        self.train_steps = 0
        # static buffers of the captured vector step (HIP graphs on a GPU; eager otherwise).
        # On a GPU a vector step is 4-5 launches: [pack + Q forward with the masked argmax
        # fused | the env's random policy], the env step, and lb_replay_add (replay write,
        # obs <- next obs, episode sums), whose slot word alternates between two graphs.
        self.use_graphs = self.device.type == "cuda"
        self._parity = 0
        self._graph = None
        self._q = torch.zeros((self.num_envs, env.observation_space.shape[0]), device=self.device)
        self._qfrag = fused.frag_buffer(self.device) if self.use_graphs else None
        self._obs = torch.zeros_like(self._next_obs)
        self._masks = torch.ones((self.num_envs, env.action_space.n), dtype=torch.bool, device=self.device)
        # device RNG (GPU): explore decisions and replay samples drawn by kernels, keyed by
        # this 64-bit seed and the vector step counter held in two alternating device words
        self.device_rng = self.use_graphs and (True if device_rng is None else bool(device_rng))
        self.period_graph = self.device_rng and self.train_graph and (True if period_graph is None
                                                                      else bool(period_graph))
        self._rng_seed = (int(seed) * 0x9E3779B97F4A7C15 + 0x632BE59BD9B4E019) & ((1 << 64) - 1)
        self._vstep_pp = torch.zeros(2, dtype=torch.int64, device=self.device)
        self._explore_flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._base_adds = torch.zeros(1, dtype=torch.int64, device=self.device)
        self._ex = [None, None]  # LBDQNExploreC per parity (kept alive: graphs hold their pointers' targets)
        self._ex_same = [None, None]
        # a train period's vector steps in one launch where the env allows it (lb_dqn_steps)
        self.multi_step = (os.environ.get("LBK8S_DQN_MULTISTEP", "1") == "1") if multi_step is None else bool(multi_step)
        self._dqn_sync = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._pgraphs = {}
        self._pgraph_slope = None
        # consecutive train periods replayed as ONE graph (single rank): the host's per-period
        # work (a graph launch, the replay-slot mirror, the train-step bookkeeping) otherwise
        # left the GPU idle between periods (config 5: ~85 us per 10-step period)
        self.periods_per_graph = max(1, int(os.environ.get("LBK8S_DQN_PERIODS_PER_GRAPH", "4")))
        self._tstatic = None
        # the target network's image, packed when the target changes (every
        # target_network_frequency steps), outside the captured periods
        self._tfrag = fused.frag_buffer(self.device) if self.device_rng else None
        # the q network's training-backward image, packed with its forward image at the start
        # of every train period (lb_ds_pack_pair) and pinned for the run
        self._qbfrag = fused.bwd_frag_buffer(self.device) if self.device_rng else None
        self._one = None

    def select_actions(self, obs, masks, epsilon):
        if random.random() < epsilon:  # one draw decides exploration for every env (:127)
            return self._explore_actions(masks).long()
        with torch.no_grad():
            q = torch.where(masks, fused.q_forward(self.q_network, obs), torch.full((), HUGE_NEG, device=obs.device))
        return torch.argmax(q, dim=1)

    def _explore_actions(self, masks):
        """np.random.choice(valid_actions) per env (:128-131).  Masks are always all True
        (:808-821), so this is a uniform action: the env's Philox draw (D_ACT)."""
        return self.env.policy("random", out=self._act)

    def _vector_step(self, obs, masks, explore, parity=0):
        """One vector step on the device: actions, fused env step, replay write, episode
        sums, obs <- next obs.  No host sync; graph-capturable."""
        env = self.env
        if explore:
            self._explore_actions(masks)
        elif self.use_graphs:
            fused.q_argmax_graphable(self.q_network, obs, masks, self._act, self._qfrag)
        else:
            with torch.no_grad():
                q = torch.where(masks, fused.q_forward(self.q_network, obs), torch.full((), HUGE_NEG, device=obs.device))
                self._act.copy_(torch.argmax(q, dim=1))
        env.step_device(self._act, obs_out=self._next_obs, reward_out=self._rew, done_out=self._done_u8)
        if self.use_graphs:
            self.rb.add_fused(obs, self._next_obs, self._act, self._rew, self._done_u8, env.ep_stats,
                              self._ep_sum, self._ep_cnt, parity)
            return
        dones = self._done_u8.float()
        self._ep_sum += env.ep_stats[:, 0] * dones
        self._ep_cnt += dones
        self.rb.add_device(obs, self._next_obs, self._act, self._rew, dones)
        obs.copy_(self._next_obs)

    # ---- device-RNG mode -----------------------------------------------------------------
    def _set_schedule(self, total_timesteps):
        """lb_dqn_explore structs for this learn() call (linear_schedule's slope, :32-34)."""
        from ._native import LBDQNExploreC
        duration = self.exploration_fraction * total_timesteps
        slope = (self.end_e - self.start_e) / duration
        base = self._vstep_pp.data_ptr()
        for parity in (0, 1):
            self._ex[parity] = LBDQNExploreC(self.start_e, slope, self.end_e, self._rng_seed, base + 8 * parity,
                                             base + 8 * (1 - parity), self._explore_flag.data_ptr())
            # (lb_dqn_steps over an even number of steps: the counter ends in the word it started in)
            self._ex_same[parity] = LBDQNExploreC(self.start_e, slope, self.end_e, self._rng_seed, base + 8 * parity,
                                                  base + 8 * parity, self._explore_flag.data_ptr())
        return slope

    def _vector_step_dev(self, obs, masks, parity):
        """One vector step with the explore decision on the device: [random actions | greedy
        actions from the packed image] in one launch (lb_dqn_act), the env step, lb_replay_add.
        The q image (self._qfrag) is packed by the caller."""
        env, pp = self.env, self.rb.pos_pp.data_ptr()
        # (lb_dqn_step: the three in one launch at config 5's shape, bit for bit)
        env.dqn_step(self._qfrag, obs, masks, self._ex[parity], self._act, self._next_obs, self._rew, self._done_u8,
                     self.rb, pp + 8 * parity, pp + 8 * (1 - parity), self._ep_sum, self._ep_cnt)

    def _vector_steps_dev(self, obs, masks, parity, n):
        """n vector steps from `parity`: one lb_dqn_steps launch where the env's shape has the
        one-launch step (the Q network is fixed within a period), else n _vector_step_dev."""
        env, pp = self.env, self.rb.pos_pp.data_ptr()
        if 1 < n <= DQN_STEPS_MAX and self.multi_step and env.dqn_steps_supported(obs.shape[1]):
            end = parity ^ (n & 1)
            ex = self._ex[parity] if end != parity else self._ex_same[parity]
            env.dqn_steps(n, self._qfrag, obs, masks, ex, self._act, self._next_obs, self._rew, self._done_u8,
                          self.rb, pp + 8 * parity, pp + 8 * end, self._ep_sum, self._ep_cnt, self._dqn_sync)
            return
        for i in range(n):
            self._vector_step_dev(obs, masks, parity ^ (i & 1))

    def _sample_dev(self, parity):
        """lb_replay_sample into the train step's fixed buffers; the counter is the vector step
        word of `parity` (the step count after the period's last step)."""
        rb, B = self.rb, self.batch_size
        if self._tstatic is None:
            self._alloc_tstatic()
        o, a, no, d, r = self._tstatic
        vp = self._vstep_pp.data_ptr() + 8 * parity
        _native.check(_native.lib().lb_replay_sample(
            self.num_envs, int(rb.obs[0, 0].numel()), rb.size, B, self._rng_seed ^ 0x5851F42D4C957F2D, vp,
            self._base_adds.data_ptr(), rb.obs.data_ptr(), rb.next_obs.data_ptr(), rb.actions.data_ptr(),
            rb.rewards.data_ptr(), rb.dones.data_ptr(), o.data_ptr(), no.data_ptr(), a.data_ptr(), r.data_ptr(),
            d.data_ptr(), torch.cuda.current_stream(self.device).cuda_stream))

    def _period_body(self, obs, masks, n, train, parity):
        """n vector steps from `parity` then (train) the sample and the train step; returns
        the graphs' split point for the all_reduce (multi-rank) via self._period_split."""
        # (with the train step, its backward's image of the same weights in the same launch)
        fused.pack_q_into(self.q_network, self._qfrag, self._qbfrag if train else None)
        self._vector_steps_dev(obs, masks, parity, n)
        if train:
            self._sample_dev(parity ^ (n & 1))
            self._tloss = self._train_backward(*self._tstatic)

    def _reps(self):
        return 1 if self._multi else self.periods_per_graph

    def _build_period_graphs(self, obs, masks):
        """Capture the period graphs: keys (n, train, parity, reps) for n in {1, train_frequency};
        reps > 1: that many consecutive train periods in one graph (single rank)."""
        F = self.train_frequency
        if self._tstatic is None:
            self._alloc_tstatic()
        # only the torch part needs a warm-up (its allocations); the vector steps and the
        # sample are native launches on fixed buffers, captured without running them, so the
        # env, the replay and the step counter are untouched and a graphed learn() follows
        # the same trajectory as an eager one
        self._train_warmup()
        graphs = {}
        keys = {(1, False, 1), (F, False, 1), (F, True, 1), (F, True, self._reps())}
        for n, train, reps in sorted(keys):
            for parity in (0, 1):
                self._tloss = None
                ga = torch.cuda.CUDAGraph()
                with torch.cuda.graph(ga):
                    p = parity
                    for _ in range(reps):
                        self._period_body(obs, masks, n, train, p)
                        if train and not self._multi:
                            self._train_apply()
                        p ^= n & 1
                gs = (ga,)
                if train and self._multi:
                    gb = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(gb):
                        self._train_apply()
                    gs = (ga, gb)
                # (each graph writes its own loss tensor: the last period's)
                graphs[n, train, parity, reps] = (gs, self._tloss)
        return graphs

    def _chunk(self, g, total_timesteps):
        """How many consecutive train periods from step g (a period start) one graph replays:
        periods_per_graph when each is a whole train period and none but the last ends on a
        target-network update or holds a logged step, else 1."""
        F, R = self.train_frequency, self._reps()
        if R == 1:
            return 1
        for r in range(R):
            g0 = g + r * F
            last = g0 + F - 1
            if not (g0 % F == 1 % F and g0 + F <= total_timesteps and last > self.learning_starts and last % F == 0):
                return 1
            if r < R - 1 and (last % self.target_network_frequency == 0
                              or any(s % 1000 == 0 or s == total_timesteps - 1 for s in range(g0, last + 1))):
                return 1
        return R

    def _alloc_tstatic(self):
        B, rb = self.batch_size, self.rb
        obs_shape = tuple(rb.obs.shape[2:])
        self._tstatic = (torch.zeros((B,) + obs_shape, device=self.device),
                         torch.zeros((B, 1), dtype=torch.long, device=self.device),
                         torch.zeros((B,) + obs_shape, device=self.device),
                         torch.zeros((B, 1), device=self.device), torch.zeros((B, 1), device=self.device))

    def _train_warmup(self):
        """Two train steps on a side stream (grads, Adam state, workspaces allocated before a
        capture), then the parameters and the Adam state (moments and step counter) restored
        to their values before the warm-up: nothing is drawn.  (The period graphs are rebuilt
        whenever a learn() changes the exploration slope; training continues from the same
        optimizer state.)"""
        params = list(self.q_network.parameters())
        snap = [p.detach().clone() for p in params]
        opt_snap = self._snapshot_optimizer()
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(2):
                self._train_backward(*self._tstatic)
                self._allreduce()
                self._train_apply()
        torch.cuda.current_stream(self.device).wait_stream(side)
        with torch.no_grad():
            for p, q in zip(params, snap):
                p.copy_(q)
        self._restore_optimizer(opt_snap)
        fused.invalidate(self.q_network)

    def _after_train(self, global_step):
        fused.invalidate(self.q_network)
        self.train_steps += 1
        if global_step % self.target_network_frequency == 0:
            with torch.no_grad():
                for tp, qp in zip(self.target_network.parameters(), self.q_network.parameters()):
                    tp.copy_(self.tau * qp + (1.0 - self.tau) * tp)
            fused.invalidate(self.target_network)
            fused.pack_q_into(self.target_network, self._tfrag)

    def _learn_device(self, total_timesteps):
        """learn() with device RNG: one graph replay per train period (period_graph) or the
        same kernels eagerly."""
        env = self.env
        start = time.time()
        obs, masks = self._obs, self._masks
        slope = self._set_schedule(total_timesteps)
        env.reset()
        obs.copy_(env.obs)
        # both images are pinned for the run: the q image is packed at the start of every
        # period (the train step's forward reuses it: no repack inside the period), the
        # target's when the target changes
        fused.pack_q_into(self.q_network, self._qfrag, self._qbfrag)
        fused.pack_q_into(self.target_network, self._tfrag)
        fused.pin(self.q_network, self._qfrag)
        fused.pin(self.target_network, self._tfrag)
        fused.pin_backward(self.q_network, self._qbfrag)
        try:
            return self._learn_device_loop(total_timesteps, start, slope)
        finally:
            fused.pin(self.q_network, None)
            fused.pin(self.target_network, None)
            fused.pin_backward(self.q_network, None)
            fused.invalidate(self.q_network)
            fused.invalidate(self.target_network)

    def prepare(self, total_timesteps):
        """Capture the period graphs of a learn(total_timesteps) (its exploration slope) without
        running a step: a following learn() with the same total replays them instead of
        capturing them inside its own wall time (a one-time cost; benchmarks call this first)."""
        if not self.period_graph:
            return
        slope = self._set_schedule(total_timesteps)
        if self._pgraphs and self._pgraph_slope == slope:
            return
        fused.pin(self.q_network, self._qfrag)
        fused.pin(self.target_network, self._tfrag)
        fused.pin_backward(self.q_network, self._qbfrag)
        try:
            self._pgraphs = self._build_period_graphs(self._obs, self._masks)
            self._pgraph_slope = slope
        finally:
            fused.pin(self.q_network, None)
            fused.pin(self.target_network, None)
            fused.pin_backward(self.q_network, None)
            fused.invalidate(self.q_network)
            fused.invalidate(self.target_network)

    def _learn_device_loop(self, total_timesteps, start, slope):
        env = self.env
        obs, masks = self._obs, self._masks
        if self.period_graph and (not self._pgraphs or self._pgraph_slope != slope):
            # (captured, not run: the env, replay and counters are untouched)
            self._pgraphs = self._build_period_graphs(obs, masks)
            self._pgraph_slope = slope
        # the replay's device slot lives in pos_pp[parity]: after a learn() with an odd number
        # of vector steps it is in word 1, so move it to word 0 with the parity (a second
        # learn() would otherwise rewrite the last transition and run one slot behind the
        # host's pos)
        if self._parity:
            self.rb.pos_pp[0].copy_(self.rb.pos_pp[1])
        self._parity = 0
        self._vstep_pp.zero_()
        self._base_adds.fill_(self.rb.size if self.rb.full else self.rb.pos)
        F = self.train_frequency
        loss = None
        g = 0
        while g < total_timesteps:
            n = F if (g % F == 1 % F and g + F <= total_timesteps) else 1
            last = g + n - 1
            train = last > self.learning_starts and last % F == 0
            if self.period_graph:
                reps = self._chunk(g, total_timesteps) if (n == F and train) else 1
                hit = self._pgraphs.get((n, train, self._parity, reps))
                if hit is None:  # (a step count the graphs do not hold)
                    n, last, reps = 1, g, 1
                    train = last > self.learning_starts and last % F == 0
                    hit = self._pgraphs[n, train, self._parity, reps]
                gs, tloss = hit
                gs[0].replay()
                if len(gs) > 1:
                    self._allreduce()  # eager collective on the current stream, between the two graphs
                    gs[1].replay()
                if train:
                    loss = tloss
                for _ in range(reps - 1):  # (the chunk's earlier periods: the host mirror)
                    for _ in range(n):
                        self._parity ^= 1
                        self.rb.advance_host()
                    self._after_train(last)
                    g, last = g + n, last + n
            else:
                self._period_body(obs, masks, n, train, self._parity)
                if train:
                    if self._multi and not self.train_graph:
                        allreduce_gradients(self.q_network)
                    else:
                        self._allreduce()
                    self._train_apply()
                    loss = self._tloss
            for _ in range(n):
                self._parity ^= 1
                self.rb.advance_host()
            if train:
                self._after_train(last)
            marks = [s for s in range(g, last + 1) if s % 1000 == 0 or s == total_timesteps - 1]
            if marks:
                # (logged at the 1000-step boundary inside the period, as the host loop logs it;
                # the returns flushed are those of the whole period)
                self._flush_returns()
                now = time.time()
                for s in marks:  # one line per mark, as the host loop writes them
                    eps = linear_schedule(self.start_e, self.end_e, self.exploration_fraction * total_timesteps, s)
                    self.log_fn(dict(global_step=s, epsilon=eps, sps=(s + 1) / (now - start),
                                     loss=None if loss is None else loss.item(),
                                     ep_return=self.episode_returns[-1] if self.episode_returns else float("nan")))
            g = last + 1
        return self

    def _build_graphs(self, obs, masks):
        """The four vector-step variants (explore or not, slot word 0 or 1) captured once as
        HIP graphs.  The warm-up steps run on a side stream before capture; the caller
        resets afterwards."""
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for explore in (False, True):
                for parity in (0, 1):
                    self._vector_step(obs, masks, explore, parity)
        torch.cuda.current_stream(self.device).wait_stream(side)
        graphs = {}
        for explore in (False, True):
            for parity in (0, 1):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self._vector_step(obs, masks, explore, parity)
                graphs[explore, parity] = g
        return graphs

    def _train_backward(self, obs, actions, next_obs, dones, rewards):
        """dqn_deepset.py:180-190: TD loss and its gradients; with several ranks the gradients
        end packed in the flat bucket that the all_reduce averages."""
        loss, _, _ = dqn_loss(self.q_network, self.target_network, obs, actions, next_obs, rewards, dones,
                              self.gamma)
        # (also inside a captured step: autograd then allocates the gradients from the graph's
        # pool, at the same addresses every replay, and no zero fill + accumulate per parameter
        # is recorded)
        self.optimizer.zero_grad(set_to_none=True)
        # (the seed gradient from a fixed tensor: loss.backward() fills a new one each step)
        if self._one is None or self._one.device != loss.device:
            self._one = fused_train.unit_seed(loss.device, loss.dtype)
        loss.backward(self._one)
        if self._multi and self.train_graph:
            torch.cat([p.grad.reshape(-1) for p in self.q_network.parameters()], out=self._gflat)
        return loss

    def _train_apply(self):
        if self._multi and self.train_graph:
            self._gflat /= torch.distributed.get_world_size()
            off = 0
            for p in self.q_network.parameters():
                n = p.numel()
                p.grad.copy_(self._gflat[off:off + n].view_as(p))
                off += n
        self.optimizer.step()

    def _capture_train(self):
        """Capture the train step on fixed sample buffers: one graph on one rank, two graphs
        around the gradient all_reduce on several (as PPO's minibatch step).  The warm-up
        steps are undone (parameters and Adam state restored) and draw nothing from the
        sampling generator, so a graphed run trains exactly as an eager one."""
        B, rb = self.batch_size, self.rb
        obs_shape = tuple(rb.obs.shape[2:])
        self._tstatic = (torch.zeros((B,) + obs_shape, device=self.device),
                         torch.zeros((B, 1), dtype=torch.long, device=self.device),
                         torch.zeros((B,) + obs_shape, device=self.device),
                         torch.zeros((B, 1), device=self.device), torch.zeros((B, 1), device=self.device))
        params = list(self.q_network.parameters())
        snap = [p.detach().clone() for p in params]
        opt_snap = self._snapshot_optimizer()
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(2):  # warm-up: allocates grads, Adam state, workspaces
                self._train_backward(*self._tstatic)
                self._allreduce()
                self._train_apply()
        torch.cuda.current_stream(self.device).wait_stream(side)
        if self._multi:
            ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(ga):
                self._tloss = self._train_backward(*self._tstatic)
            with torch.cuda.graph(gb):
                self._train_apply()
            self._tgraphs = (ga, gb)
        else:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._tloss = self._train_backward(*self._tstatic)
                self._train_apply()
            self._tgraphs = (g,)
        with torch.no_grad():
            for p, q in zip(params, snap):
                p.copy_(q)
        self._restore_optimizer(opt_snap)
        fused.invalidate(self.q_network)

    def _snapshot_optimizer(self):
        """Copies of the Adam state tensors (moments, step) by parameter, before a warm-up."""
        return {id(p): {k: v.detach().clone() for k, v in st.items() if isinstance(v, torch.Tensor)}
                for p, st in self.optimizer.state.items()}

    def _restore_optimizer(self, saved):
        """Undo a warm-up's optimizer steps: state that existed before it gets its values
        back, state the warm-up created (a fresh optimizer) is zeroed (step 0, zero moments)."""
        with torch.no_grad():
            for p, st in self.optimizer.state.items():
                old = saved.get(id(p), {})
                for k, v in st.items():
                    if isinstance(v, torch.Tensor):
                        if k in old:
                            v.copy_(old[k])
                        else:
                            v.zero_()

    def _allreduce(self):
        if self._multi and self.train_graph:
            lbdist.all_reduce_sum(self._gflat)

    def train_step(self, global_step):
        if self.train_graph:
            if self._tgraphs is None:
                self._capture_train()
            self.rb.sample_into(self.batch_size, self._tstatic)
            self._tgraphs[0].replay()
            if len(self._tgraphs) > 1:
                self._allreduce()  # eager collective on the current stream, between the two graphs
                self._tgraphs[1].replay()
            loss = self._tloss
        else:
            loss = self._train_backward(*self.rb.sample(self.batch_size))
            allreduce_gradients(self.q_network)
            self._train_apply()
        # the fused forward's cached weight image of the q network is stale now: neither a
        # replayed Adam step nor torch's fused Adam kernel moves the version counters it keys on
        fused.invalidate(self.q_network)
        self.train_steps += 1
        if global_step % self.target_network_frequency == 0:
            # (dqn_deepset.py:199-203) in place on the parameters themselves, so their version
            # counters move and the fused forward's cached weight image of the target is rebuilt
            # (writes through .data would leave that image stale)
            with torch.no_grad():
                for tp, qp in zip(self.target_network.parameters(), self.q_network.parameters()):
                    tp.copy_(self.tau * qp + (1.0 - self.tau) * tp)
            fused.invalidate(self.target_network)
        return loss

    def learn(self, total_timesteps: int = 500000):
        env = self.env
        if self.device_rng and not env.monitor:
            return self._learn_device(total_timesteps)
        start = time.time()
        env.reset()
        obs, masks = self._obs, self._masks  # fixed buffers: the captured graphs use them
        obs.copy_(env.obs)
        graphs = None
        if self.use_graphs:
            if self._graph is None:
                self._graph = self._build_graphs(obs, masks)
                # the warm-up / capture steps advanced envs, replay and accumulators: restart
                env.reset()
                obs.copy_(env.obs)
                self.rb.clear()
                self._parity = 0
                self._ep_sum.zero_()
                self._ep_cnt.zero_()
            graphs = self._graph
        loss = None
        for global_step in range(total_timesteps):
            eps = linear_schedule(self.start_e, self.end_e, self.exploration_fraction * total_timesteps, global_step)
            explore = random.random() < eps  # one draw decides exploration for every env (:127)
            if graphs is not None:
                graphs[explore, self._parity].replay()
            else:
                self._vector_step(obs, masks, explore, self._parity)
            env.record_episodes(self._done_u8, self._rew, self._act)  # VecMonitor file, if any
            self._parity ^= 1
            self.rb.advance_host()
            if global_step > self.learning_starts and global_step % self.train_frequency == 0:
                loss = self.train_step(global_step)
            if global_step % 1000 == 0 or global_step == total_timesteps - 1:
                self._flush_returns()
                self.log_fn(dict(global_step=global_step, epsilon=eps, sps=(global_step + 1) / (time.time() - start),
                                 loss=None if loss is None else loss.item(),
                                 ep_return=self.episode_returns[-1] if self.episode_returns else float("nan")))
        return self

    def _flush_returns(self):
        self.env.flush_monitor()
        mean, _ = lbdist.mean_episode_return(self._ep_sum, self._ep_cnt)  # over every rank
        if mean is not None:
            self.episode_returns.append(mean)
        self._ep_sum.zero_()
        self._ep_cnt.zero_()

    def predict(self, obs, masks=None):
        with torch.no_grad():
            x = torch.as_tensor(obs, dtype=torch.float32, device=self.device)
            m = None if masks is None else torch.as_tensor(masks, dtype=torch.bool, device=self.device)
            return self.q_network.get_action(x, m, deterministic=True)

    def save(self, path):
        torch.save(self.q_network.state_dict(), path)

    def load(self, path):
        self.q_network.load_state_dict(torch.load(path, map_location=self.device, weights_only=True))

"""GPU-resident PPO for the deep-sets agent.

Restates envs/ppo_deepset.py (CleanRL PPO, :53-300) on device tensors end to end:
rollout storage (T, B, ...) filled by LBVecEnv.step_device (obs written straight into
the storage slot, no host copies), GAE (:192-205), flattened minibatches, clipped policy
and value losses, entropy bonus, advantage normalisation per minibatch, clip_grad_norm,
Adam(eps=1e-5) (:216-267).  Hyper-parameter names and defaults are the reference's.
Reference quirk kept: actions are sampled WITHOUT masks during the rollout (:169; the
masks are all True anyway, :808-821) and the stored masks are used in the update.

Multi-GPU: one process per GPU, each with its own envs (LBVecEnv env_id_offset); the
gradients are averaged with one all_reduce per optimizer step (RCCL over xGMI) and the
logged episode return is the mean over every rank's finished episodes.

The minibatch step (loss, fused forward/backward, clip_grad_norm, Adam) is captured once
as HIP graphs and replayed per minibatch: ~200 launches per minibatch otherwise leave the
GPU waiting on the host between the fused kernels.  With several ranks the step is two
graphs — loss/backward ending in the gradients packed into one flat bucket, then
unpack/average + clip + Adam — with the bucket's all_reduce issued between them on the
same stream (the collective stays outside the captures, so any backend works).  The
capture's warm-up steps are undone (parameters restored, Adam state zeroed), so the graph
path computes the same update as the eager one.
"""
import os
import time
from typing import Optional

import torch
from torch import nn, optim

from . import dist as lbdist
from . import fused, fused_train
from .deepsets import DeepSetAgent


def ppo_loss(agent, obs, actions, logprobs_old, masks, advantages, returns, values_old,
             clip_coef=0.2, ent_coef=0.01, vf_coef=0.5, norm_adv=True, clip_vloss=True):
    """One minibatch of ppo_deepset.py:227-263 -> (loss, pg_loss, v_loss, entropy, approx_kl, clipfrac).

    On a HIP device the deep-sets forward/backward are the fused training kernels and the
    loss head (log-softmax, ratio, clipped losses, entropy and their gradients) is one
    launch (fused_train.ppo_head); elsewhere, the same ops as the reference in torch."""
    from . import fused_train
    if (obs.is_cuda and torch.is_grad_enabled() and fused_train.supported(agent.actor.net, obs)
            and (masks is None or masks.shape[-1] == obs.shape[1])):
        logits, newvalue = agent.actor_critic(obs)
        adv = advantages
        if norm_adv:
            adv = (adv - adv.mean()) / (adv.std() + 1e-8)
        loss, st = fused_train.ppo_head(logits, newvalue.view(-1), masks, actions, logprobs_old, adv, returns,
                                        values_old, clip_coef, ent_coef, vf_coef, clip_vloss)
        return loss, st[0], 0.5 * st[1], st[2], st[3], st[4]
    # the same Categorical ops as the reference: the actor's last Gamma term shifts every
    # logit of a set equally, so its true gradient is 0 and what autograd returns is
    # rounding noise that only an identical op sequence reproduces
    _, newlogprob, entropy, newvalue = agent.get_action_and_value(obs, actions.long(), masks)
    newvalue = newvalue.view(-1)
    logratio = newlogprob - logprobs_old
    ratio = logratio.exp()
    adv = advantages
    if norm_adv:
        adv = (adv - adv.mean()) / (adv.std() + 1e-8)
    pg_loss = torch.max(-adv * ratio, -adv * torch.clamp(ratio, 1 - clip_coef, 1 + clip_coef)).mean()
    if clip_vloss:
        v_unclipped = (newvalue - returns) ** 2
        v_clipped = values_old + torch.clamp(newvalue - values_old, -clip_coef, clip_coef)
        v_loss = 0.5 * torch.max(v_unclipped, (v_clipped - returns) ** 2).mean()
    else:
        v_loss = 0.5 * ((newvalue - returns) ** 2).mean()
    entropy_loss = entropy.mean()
    loss = pg_loss - ent_coef * entropy_loss + v_loss * vf_coef
    with torch.no_grad():
        approx_kl = ((ratio - 1) - logratio).mean()
        clipfrac = ((ratio - 1.0).abs() > clip_coef).float().mean()
    return loss, pg_loss, v_loss, entropy_loss, approx_kl, clipfrac


def compute_gae(rewards, values, dones, next_value, next_done, gamma, gae_lambda):
    """ppo_deepset.py:192-205 on (T, B) device tensors."""
    T = rewards.shape[0]
    advantages = torch.zeros_like(rewards)
    lastgaelam = torch.zeros_like(rewards[0])
    for t in reversed(range(T)):
        if t == T - 1:
            nextnonterminal = 1.0 - next_done
            nextvalues = next_value
        else:
            nextnonterminal = 1.0 - dones[t + 1]
            nextvalues = values[t + 1]
        delta = rewards[t] + gamma * nextvalues * nextnonterminal - values[t]
        lastgaelam = delta + gamma * gae_lambda * nextnonterminal * lastgaelam
        advantages[t] = lastgaelam
    return advantages, advantages + values


class PPO_DeepSets:
    def __init__(self, env, learning_rate: float = 2.5e-4, anneal_lr: bool = False, num_steps: int = 128,
                 gae: bool = True, gae_lambda: float = 0.97, gamma: float = 0.95, n_minibatches: int = 4,
                 update_epochs: int = 4, norm_adv: bool = True, clip_coef: float = 0.2,
                 clip_vloss: bool = True, ent_coef: float = 0.01, vf_coef: float = 0.5,
                 max_grad_norm: float = 0.5, target_kl: Optional[float] = None, seed: int = 1,
                 device=None, log_fn=None, num_envs=None, tensorboard_log=None, use_graphs=None):
        # num_envs / tensorboard_log: accepted for signature compatibility with
        # ppo_deepset.py:53-75 (the env's num_envs is used; there is no tensorboard writer)
        self.env = env
        self.device = torch.device(device) if device is not None else env.device
        self.num_envs = env.num_envs
        self.learning_rate, self.anneal_lr, self.num_steps = learning_rate, anneal_lr, num_steps
        self.gae, self.gae_lambda, self.gamma = gae, gae_lambda, gamma
        self.n_minibatches, self.update_epochs, self.norm_adv = n_minibatches, update_epochs, norm_adv
        self.clip_coef, self.clip_vloss, self.ent_coef, self.vf_coef = clip_coef, clip_vloss, ent_coef, vf_coef
        self.max_grad_norm, self.target_kl, self.seed = max_grad_norm, target_kl, seed
        self.batch_size = int(self.num_envs * num_steps)
        self.minibatch_size = int(self.batch_size // n_minibatches)
        self.log_fn = log_fn or (lambda d: None)
        torch.manual_seed(seed)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)
        self.agent = DeepSetAgent(env).to(self.device)
        self._multi = lbdist.is_multi()
        if self._multi:
            lbdist.broadcast_parameters(self.agent)  # replicas start from rank 0's weights
        # flat gradient bucket of the all_reduce (one collective per optimizer step)
        self._gflat = torch.zeros(sum(p.numel() for p in self.agent.parameters()), device=self.device) \
            if self._multi else None
        if use_graphs is None:
            use_graphs = self.device.type == "cuda"
        # a captured step needs equal minibatches and a device-side Adam step / lr
        self.use_graphs = bool(use_graphs) and self.batch_size % self.minibatch_size == 0
        if self.use_graphs:
            self._lr = torch.tensor(float(learning_rate), device=self.device)
            # torch's fused (single multi-tensor kernel) Adam: fewer launches per captured step
            self.optimizer = optim.Adam(self.agent.parameters(), lr=self._lr, eps=1e-5, capturable=True,
                                        fused=os.environ.get("LBK8S_FUSED_ADAM", "1") == "1")
        else:
            self.optimizer = optim.Adam(self.agent.parameters(), lr=learning_rate, eps=1e-5)
        self._mb_graphs = None
        T, B = num_steps, self.num_envs
        R, A = env.observation_space.shape[0], env.action_space.n
        dev = self.device
        self.obs = torch.zeros((T, B, R, 8), device=dev)
        self.actions = torch.zeros((T, B), device=dev)
        self.masks = torch.ones((T, B, A), dtype=torch.bool, device=dev)
        self.logprobs = torch.zeros((T, B), device=dev)
        self.rewards = torch.zeros((T, B), device=dev)
        self.dones = torch.zeros((T, B), device=dev)
        self.values = torch.zeros((T, B), device=dev)
        self._last_obs = torch.zeros((B, R, 8), device=dev)  # obs after the last rollout step
        self._act = torch.zeros(B, dtype=torch.int32, device=dev)
        self._done_u8 = torch.zeros(B, dtype=torch.uint8, device=dev)
        self.episode_returns = []
        self._ep_sum = torch.zeros((), dtype=torch.float64, device=dev)
        self._ep_cnt = torch.zeros((), dtype=torch.float64, device=dev)
        # the rollout's categorical draws: T x B uniforms drawn in one call per rollout, the
        # samples by inverse CDF (no multinomial launch chain or host-synchronising check per
        # step).  Capturing the T steps as one HIP graph was measured (config 4: 19.5 ms per
        # rollout either way): the rollout is GPU-bound, so it runs eagerly.
        self._u = torch.zeros((T, B), device=dev)

    def _rollout_body(self, next_done):
        """The T vector steps on the storage buffers (no host sync, no RNG call: the uniforms
        are drawn before).  Returns the done flags after the last step."""
        env = self.env
        T = self.num_steps
        next_obs = self.obs[0]
        for step in range(T):
            self.dones[step] = next_done
            action, logprob, value = self.agent.act(next_obs, uniforms=self._u[step])  # no masks (:169)
            self.values[step] = value
            self.actions[step] = action.float()
            self.logprobs[step] = logprob
            self._act.copy_(action)
            # the env writes the next observation straight into the next storage slot
            next_obs = self.obs[step + 1] if step + 1 < T else self._last_obs
            env.step_device(self._act, obs_out=next_obs, reward_out=self.rewards[step], done_out=self._done_u8)
            env.record_episodes(self._done_u8, self.rewards[step], self._act)  # VecMonitor file, if any
            next_done = self._done_u8.float()
            # finished-episode returns accumulate on the device (no per-step host sync)
            self._ep_sum += (env.ep_stats[:, 0] * next_done).sum()
            self._ep_cnt += next_done.sum()
        return next_done

    def rollout(self, next_obs, next_done):
        """Fill the (T, B) storage; returns the obs/done that follow the last step."""
        env = self.env
        if next_obs.data_ptr() != self.obs[0].data_ptr():
            self.obs[0].copy_(next_obs)
        torch.rand(self._u.shape, generator=self.gen, device=self.device, out=self._u)
        next_done = self._rollout_body(next_done)
        next_obs = self._last_obs
        env.flush_monitor()
        mean, _ = lbdist.mean_episode_return(self._ep_sum, self._ep_cnt)  # over every rank
        if mean is not None:
            self.episode_returns.append(mean)
        self._ep_sum.zero_()
        self._ep_cnt.zero_()
        return next_obs, next_done

    def _mb_backward(self, obs, actions, logprobs, masks, adv, ret, val):
        """Loss and gradients of one minibatch; with several ranks the gradients end packed
        in the flat bucket that the all_reduce averages."""
        out = ppo_loss(self.agent, obs, actions, logprobs, masks, adv, ret, val,
                       self.clip_coef, self.ent_coef, self.vf_coef, self.norm_adv, self.clip_vloss)
        # (also inside a captured step: autograd then allocates the gradients from the graph's
        # pool, at the same addresses every replay, and no zero fill + accumulate per parameter
        # is recorded)
        self.optimizer.zero_grad(set_to_none=True)
        # (a fixed unit seed: the fused loss head returns its saved gradients as they are)
        seed = getattr(self, "_seed1", None)
        if seed is None or seed.device != out[0].device or seed.dtype != out[0].dtype:
            seed = self._seed1 = fused_train.unit_seed(out[0].device, out[0].dtype)
        out[0].backward(seed)
        if self._multi:
            torch.cat([p.grad.reshape(-1) for p in self.agent.parameters()], out=self._gflat)
        return out

    def _mb_apply(self):
        """Averaged gradients (several ranks) -> clip_grad_norm -> Adam."""
        if self._multi:
            self._gflat /= torch.distributed.get_world_size()
            off = 0
            for p in self.agent.parameters():
                n = p.numel()
                p.grad.copy_(self._gflat[off:off + n].view_as(p))
                off += n
        nn.utils.clip_grad_norm_(self.agent.parameters(), self.max_grad_norm)
        self.optimizer.step()

    def _allreduce(self):
        if self._multi:
            lbdist.all_reduce_sum(self._gflat)

    def _minibatch_step(self, *mb):
        out = self._mb_backward(*mb)
        self._allreduce()
        self._mb_apply()
        return out

    def _capture(self, src, mb):
        """Capture one minibatch step on static buffers (filled from minibatch `mb`): one
        graph on one rank, two graphs around the gradient all_reduce on several."""
        self._static = [torch.empty((self.minibatch_size,) + t.shape[1:], dtype=t.dtype, device=t.device)
                        for t in src]
        for d, t in zip(self._static, src):
            torch.index_select(t, 0, mb, out=d)
        params = list(self.agent.parameters())
        snap = [p.detach().clone() for p in params]
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(2):  # warm-up: allocates grads, Adam state, workspaces
                self._minibatch_step(*self._static)
        torch.cuda.current_stream(self.device).wait_stream(side)
        if self._multi:
            ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(ga):
                self._static_out = self._mb_backward(*self._static)
            with torch.cuda.graph(gb):
                self._mb_apply()
            graphs = (ga, gb)
        else:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._static_out = self._minibatch_step(*self._static)
            graphs = (g,)
        with torch.no_grad():  # undo the warm-up steps
            for p, q in zip(params, snap):
                p.copy_(q)
            for st in self.optimizer.state.values():
                for v in st.values():
                    if isinstance(v, torch.Tensor):
                        v.zero_()
        self._mb_graphs = graphs

    def _replay(self):
        if len(self._mb_graphs) == 1:
            self._mb_graphs[0].replay()
            return
        self._mb_graphs[0].replay()
        self._allreduce()  # eager collective on the current stream, between the two graphs
        self._mb_graphs[1].replay()

    def update(self, next_obs, next_done):
        with torch.no_grad():
            next_value = self.agent.get_value(next_obs).reshape(1, -1)
            advantages, returns = compute_gae(self.rewards, self.values, self.dones, next_value, next_done,
                                              self.gamma, self.gae_lambda)
        R = self.obs.shape[2]
        b_obs = self.obs.reshape(-1, R, 8)
        b_logprobs = self.logprobs.reshape(-1)
        b_actions = self.actions.reshape(-1)
        b_masks = self.masks.reshape(-1, self.masks.shape[-1])
        b_adv, b_ret, b_val = advantages.reshape(-1), returns.reshape(-1), self.values.reshape(-1)
        src = (b_obs, b_actions, b_logprobs, b_masks, b_adv, b_ret, b_val)
        stats = {}
        for epoch in range(self.update_epochs):
            b_inds = torch.randperm(self.batch_size, device=self.device, generator=self.gen)
            for start in range(0, self.batch_size, self.minibatch_size):
                mb = b_inds[start:start + self.minibatch_size]
                if self.use_graphs:
                    if self._mb_graphs is None:
                        self._capture(src, mb)
                    for d, t in zip(self._static, src):
                        torch.index_select(t, 0, mb, out=d)
                    self._replay()
                    out = self._static_out
                else:
                    out = self._minibatch_step(*(t[mb] for t in src))
                loss, pg, vl, ent, kl, cf = out
            if self.target_kl is not None:
                # every rank takes the same decision (one rank leaving the epoch loop early
                # would skip collectives the others still issue): the mean kl over the ranks
                kl_all = kl.detach().clone()
                if self._multi:
                    lbdist.all_reduce_sum(kl_all)
                    kl_all /= torch.distributed.get_world_size()
                if kl_all > self.target_kl:
                    break
        if self.use_graphs:
            fused.invalidate(self.agent)  # replayed Adam steps do not move the version counters
        stats.update(loss=loss.item(), pg_loss=pg.item(), v_loss=vl.item(), entropy=ent.item(),
                     approx_kl=kl.item(), clipfrac=cf.item())
        return stats

    def learn(self, total_timesteps: int = 500000):
        env = self.env
        start = time.time()
        next_obs = env.reset()
        if not isinstance(next_obs, torch.Tensor):
            next_obs = env.obs
        next_done = torch.zeros(self.num_envs, device=self.device)
        num_updates = total_timesteps // self.batch_size
        global_step = 0
        for update in range(1, num_updates + 1):
            if self.anneal_lr:
                lr = (1.0 - (update - 1.0) / num_updates) * self.learning_rate
                if self.use_graphs:
                    self._lr.fill_(lr)  # the captured Adam step reads the lr tensor
                else:
                    self.optimizer.param_groups[0]["lr"] = lr
            next_obs, next_done = self.rollout(next_obs, next_done)
            global_step += self.batch_size
            stats = self.update(next_obs, next_done)
            stats.update(update=update, global_step=global_step,
                         sps=global_step / (time.time() - start),
                         ep_return=self.episode_returns[-1] if self.episode_returns else float("nan"))
            self.log_fn(stats)
        return self

    def predict(self, obs, masks=None):
        with torch.no_grad():
            x = torch.as_tensor(obs, dtype=torch.float32, device=self.device)
            m = None if masks is None else torch.as_tensor(masks, dtype=torch.bool, device=self.device)
            return self.agent.get_action(x, m, deterministic=True)

    def save(self, path):
        torch.save(self.agent.state_dict(), path)

    def load(self, path):
        self.agent.load_state_dict(torch.load(path, map_location=self.device, weights_only=True))

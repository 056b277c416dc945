"""Deep-sets policy / value / Q networks.

Same architecture and parameter names as the reference, so `state_dict`s load either way:
  * EquivariantLayer  x -> Lambda(x) - Gamma(max over the set of x)   (no bias)
                      envs/deep_sets_agent_original.py:56-66
  * EquivariantDeepSet  Eq(C->64) ReLU Eq(64->64) ELU Eq(64->1) -> per-element logits   :69-83
  * InvariantDeepSet    psi = Eq ELU Eq ELU Eq (64), mean over the set, rho = Linear ELU
                        Linear -> V(s)                                                  :86-106
  * DeepSetAgent (actor = equivariant, critic = invariant)                              :109-145
  * DQNDeepSetAgent (one equivariant Q network)          envs/deep_sets_agent_dqn.py:10-42
Masks follow the reference: logits of invalid actions become -1e8 before the Categorical.

`DeepSetAgent.act(obs)` is the rollout entry point: on a HIP device with the fused
kernel available (lb_ds_forward in liblbk8s.so) it evaluates actor and critic in one
launch; otherwise it runs these torch modules.  Training on a HIP device
(`DeepSetAgent.get_action_and_value` / `DQNDeepSetAgent.forward` with grad enabled) runs
the fused training kernels (lbk8s/fused_train.py); on the CPU, autograd through these
modules.
"""
from typing import Optional

import torch
from torch import nn
from torch.distributions import Categorical

HUGE_NEG = -1e8


SPLITK_ROWS = 8192  # rows per partial product of a split-K weight gradient


def splitk_weight_grad(g: torch.Tensor, x: torch.Tensor, rows: int = SPLITK_ROWS) -> torch.Tensor:
    """g^T x over all leading dims, as a batch of row-chunk GEMMs plus a sum.

    A training minibatch has 51,200 sets x 65 elements = 3.3M rows against a 64 x 64
    output: one GEMM gives hipBLASLt a handful of output tiles for a 3.3M-long reduction
    (~15 TFLOP/s measured).  Chunking the rows gives ~400 independent tiles instead."""
    O, I = g.shape[-1], x.shape[-1]
    g2, x2 = g.reshape(-1, O), x.reshape(-1, I)
    M = g2.shape[0]
    S = M // rows
    if S < 2:
        return g2.t() @ x2
    m = S * rows
    gw = torch.bmm(g2[:m].view(S, rows, O).transpose(1, 2), x2[:m].view(S, rows, I)).sum(0)
    if m < M:
        gw += g2[m:].t() @ x2[m:]
    return gw


class _EquivariantFn(torch.autograd.Function):
    """Lambda(x) - Gamma(max_set x) with a hand-written backward (GPU training path).

    Same gradients as autograd through torch.max / Linear / broadcast-subtract (the pooled
    gradient goes to the index torch.max returned), in fewer, larger kernels: split-K
    weight gradients and one scatter_add for the max instead of full-size negate and
    broadcast-reduce kernels."""

    @staticmethod
    def forward(ctx, x, lam, gam):
        pooled, idx = torch.max(x, dim=1, keepdim=True)
        ctx.save_for_backward(x, lam, gam, pooled, idx)
        return torch.nn.functional.linear(x, lam) - torch.nn.functional.linear(pooled, gam)

    @staticmethod
    def backward(ctx, gy):
        x, lam, gam, pooled, idx = ctx.saved_tensors
        gy = gy.contiguous()
        gsum = gy.sum(dim=1, keepdim=True)  # (B, 1, O): gradient reaching Gamma(pooled), negated
        g_lam = splitk_weight_grad(gy, x) if ctx.needs_input_grad[1] else None
        g_gam = -(gsum.reshape(-1, gsum.shape[-1]).t() @ pooled.reshape(-1, pooled.shape[-1])) \
            if ctx.needs_input_grad[2] else None
        gx = None
        if ctx.needs_input_grad[0]:
            gx = gy @ lam
            gx.scatter_add_(1, idx, -(gsum @ gam))
        return gx, g_lam, g_gam


class EquivariantLayer(nn.Module):
    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.Gamma = nn.Linear(in_channels, out_channels, bias=False)
        self.Lambda = nn.Linear(in_channels, out_channels, bias=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # x: (batch, elements, channels); the set-wise max is broadcast back to every element.
        # torch.max (not amax): on ties the gradient goes to the first maximum, as in the
        # reference (amax would split it; ReLU outputs tie at 0 often).
        if x.is_cuda and torch.is_grad_enabled():
            return _EquivariantFn.apply(x, self.Lambda.weight, self.Gamma.weight)
        pooled, _ = torch.max(x, dim=1, keepdim=True)
        return self.Lambda(x) - self.Gamma(pooled)


class EquivariantDeepSet(nn.Module):
    def __init__(self, in_channels: int, hidden_channels: int = 64):
        super().__init__()
        self.net = nn.Sequential(
            EquivariantLayer(in_channels, hidden_channels), nn.ReLU(),
            EquivariantLayer(hidden_channels, hidden_channels), nn.ELU(),
            EquivariantLayer(hidden_channels, 1))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.net(x).squeeze(-1)  # (batch, elements)


class InvariantDeepSet(nn.Module):
    def __init__(self, in_channels: int, hidden_channels: int = 64):
        super().__init__()
        self.psi = nn.Sequential(
            EquivariantLayer(in_channels, hidden_channels), nn.ELU(),
            EquivariantLayer(hidden_channels, hidden_channels), nn.ELU(),
            EquivariantLayer(hidden_channels, hidden_channels))
        self.rho = nn.Sequential(nn.Linear(hidden_channels, hidden_channels), nn.ELU(),
                                 nn.Linear(hidden_channels, 1))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.rho(self.psi(x).mean(dim=1)).squeeze(-1)  # (batch,)


def masked_logits(logits: torch.Tensor, masks: Optional[torch.Tensor]) -> torch.Tensor:
    if masks is None:
        return logits
    return torch.where(masks, logits, torch.full_like(logits, HUGE_NEG))


def _in_channels(envs_or_shape):
    if isinstance(envs_or_shape, int):
        return envs_or_shape
    return envs_or_shape.observation_space.shape[1]


class DeepSetAgent(nn.Module):
    def __init__(self, envs, hidden_channels: int = 64):
        super().__init__()
        c = _in_channels(envs)
        self.actor = EquivariantDeepSet(c, hidden_channels)
        self.critic = InvariantDeepSet(c, hidden_channels)

    def get_value(self, x: torch.Tensor) -> torch.Tensor:
        return self.critic(x)

    def get_action(self, x, masks=None, deterministic: bool = True):
        dist = Categorical(logits=masked_logits(self.actor(x), masks))
        return dist.mode if deterministic else dist.sample()

    def actor_critic(self, x):
        """(logits, value).  Training on a HIP device (grad enabled, covered geometry) runs
        the fused training kernels (lbk8s/fused_train.py); otherwise the torch modules."""
        if x.is_cuda and torch.is_grad_enabled():
            from . import fused_train
            if fused_train.supported(self.actor.net, x):
                return fused_train.actor_critic(self, x)
        return self.actor(x), self.critic(x)

    def get_action_and_value(self, x, action=None, masks=None):
        logits, value = self.actor_critic(x)
        # validate_args=False: argument validation syncs with the host (not capturable)
        dist = Categorical(logits=masked_logits(logits, masks), validate_args=False)
        if action is None:
            action = dist.sample()
        return action, dist.log_prob(action), dist.entropy(), value

    @torch.no_grad()
    def act(self, x, masks=None, generator=None, uniforms=None):
        """Rollout step: (action, log_prob, value) with no autograd graph.  `uniforms` (B,)
        U(0,1) draws: the categorical sample by inverse CDF on them (no RNG call inside, so
        the step can be captured in a HIP graph); otherwise torch.multinomial."""
        from . import fused
        logits, value = fused.deepsets_forward(self, x)
        lg = masked_logits(logits, masks)
        logp_all = torch.log_softmax(lg, dim=-1)
        if uniforms is not None:
            c = logp_all.exp().cumsum(dim=-1)
            action = (c < uniforms[:, None] * c[:, -1:]).sum(dim=-1).clamp_(max=c.shape[-1] - 1)
        elif generator is None:
            action = torch.multinomial(logp_all.exp(), 1).squeeze(-1)
        else:
            action = torch.multinomial(logp_all.exp(), 1, generator=generator).squeeze(-1)
        return action, logp_all.gather(1, action[:, None]).squeeze(1), value


class DQNDeepSetAgent(nn.Module):
    def __init__(self, envs, hidden_channels: int = 64):
        super().__init__()
        self.q_network = EquivariantDeepSet(_in_channels(envs), hidden_channels)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda and torch.is_grad_enabled():
            from . import fused_train
            if fused_train.supported(self.q_network.net, x):
                return fused_train.actor_only(self, self.q_network.net, x)
        return self.q_network(x)

    def get_action(self, x, masks=None, deterministic: bool = True):
        dist = Categorical(logits=masked_logits(self.q_network(x), masks))
        return dist.mode if deterministic else dist.sample()


def flat_grads(module: nn.Module) -> torch.Tensor:
    return torch.cat([p.grad.reshape(-1) for p in module.parameters()])


def allreduce_gradients(module: nn.Module, group=None) -> None:
    """Average gradients over ranks with ONE collective (params are replicated).

    The deep-sets nets are 9-31k float32 parameters (37-124 KB): a single bucket, so one
    all_reduce per optimizer step (RCCL over xGMI on GPUs, gloo on CPU).
    """
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    params = [p for p in module.parameters() if p.grad is not None]
    flat = torch.cat([p.grad.reshape(-1) for p in params])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    flat /= dist.get_world_size(group)
    off = 0
    for p in params:
        n = p.numel()
        p.grad.copy_(flat[off:off + n].view_as(p.grad))
        off += n

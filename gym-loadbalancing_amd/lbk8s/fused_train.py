"""Fused deep-sets training step: lb_ds_train_forward /
lb_ds_train_backward in liblbk8s.so.

The reference trains its networks with torch autograd through the modules of
envs/deep_sets_agent_original.py:56-106 (ppo_deepset.py:227-263).  Here the equivariant
stacks run as two HIP kernels per minibatch (csrc/lbk8s_ds_train.h): a forward that keeps
the hidden activations, and a backward that walks every layer in registers (argmax of the
set-wise max recomputed from the saved activation, data gradients on f32 MFMA) and
accumulates each head's dLambda2 / dLambda1 over all rows in MFMA accumulators (no
per-row gradient reaches HBM), plus per-set vectors.  What is left — rho (a 64-wide MLP
on the set mean), the loss, and the remaining weight gradients as small GEMMs over the
sets — runs in torch:

    dLambda1 = dz1^T obs (kernel)   dGamma1 = -(sum_r dz1)^T max_set(obs)
    dLambda2 = dz2^T h1  (kernel)   dGamma2 = -(sum_r dz2)^T max_set(h1)
    actor  dLambda3 = sum_sets sum_r dlogit[r] h2[r]     dGamma3 = -(sum_r dlogit)^T max_set(h2)
    critic dLambda3 = (dmean / R)^T sum_r c2[r]          dGamma3 = -dmean^T max_set(c2)

The pooled gradient goes to the first row attaining the max, like torch.max in the
reference's autograd; the forward kernel records each layer input's set-wise max and that
row for the backward.  Covered geometry: 8 input features, 64 hidden, 1 <= R <= 257 (E <=
256 and the reject row; above 80 the forward streams the set in 32-row chunks), on a HIP
device; `supported()` says whether an input qualifies.
"""
import ctypes as C

import torch

from . import _native
from . import fused

SV = _native.LB_DS_SETVEC_FLOATS
DSV = _native.LB_DSV


def supported(actor_net, x) -> bool:
    """The training kernels take R <= LB_DS_MAX_ELEMENTS_TRAIN (257, the env's largest set);
    anything else trains through the torch modules (with their GPU custom backward,
    deepsets._EquivariantFn)."""
    return fused.ENABLED and fused._geometry_ok(actor_net, x) and x.shape[1] <= _native.LB_DS_MAX_ELEMENTS_TRAIN


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


def _pack_backward(actor_net, critic, dev):
    w, keep = fused._weights_struct(actor_net, critic)
    bfrag = torch.empty(_native.LB_DS_BWD_FLOATS, dtype=torch.float32, device=dev)
    _native.check(_native.lib().lb_ds_pack_backward(C.byref(w), bfrag.data_ptr(), _stream(dev)))
    del keep  # stream-ordered
    return bfrag


_work = {}


def _workspace(dev):
    """Per-device scratch for the backward's per-wave partial sums (stream-ordered reuse)."""
    w = _work.get(dev)
    if w is None:
        w = _work[dev] = torch.empty(_native.LB_DS_WORKSPACE_FLOATS, dtype=torch.float32, device=dev)
    return w


def _vec(setvec, name, n=64):
    o = DSV[name]
    return setvec[:, o:o + n]


SET_CHUNK = 512  # sets per partial product of a reduction over the sets
# up to this many sets the small weight gradients are one lb_ds_set_grads launch (the DQN's
# 128-set step: it replaces three GEMMs, two reductions and their fill / negation kernels);
# above, the chunked GEMMs of _over_sets
SET_GRADS_MAX_SETS = 512


def _over_sets(a, b, alpha=1.0):
    """alpha a^T b for a (S, M), b (S, N): a reduction over S sets, split into chunk GEMMs
    plus a sum so hipBLASLt gets ~S/512 independent tiles instead of one or two (a
    51,200-long K with a 64 x 64 output ran on two workgroups: 230 us; chunked: a few us).
    alpha = -1 gives the Gamma gradients' sign in the GEMM itself (no negation kernel)."""
    S = a.shape[0]
    n = S // SET_CHUNK
    z = a.new_empty(())  # (beta = 0: the input is ignored)
    if n < 2:
        return torch.addmm(z, a.t(), b, beta=0, alpha=alpha)
    m = n * SET_CHUNK
    out = torch.baddbmm(z, a[:m].reshape(n, SET_CHUNK, -1).transpose(1, 2), b[:m].reshape(n, SET_CHUNK, -1),
                        beta=0, alpha=alpha).sum(0)
    if m < S:
        out.addmm_(a[m:].t(), b[m:], alpha=alpha)
    return out


OS_SPAN = _native.LB_DS_OVER_SETS_SPAN  # lb_ds_over_sets' sets per partial sum
_os_work = {}


def sums_over_sets(jobs, S, dev):
    """lb_ds_over_sets: for each job (a, b, scale) with a (S, M) or None (a plain sum of b's rows)
    and b (S, N) -- 2-D views with unit column stride -- the (M, N) tensor scale * a^T b, all jobs in
    two launches (an MFMA partial sum per OS_SPAN-set span, then the spans added in order)."""
    outs, cjobs, row = [], [], 0
    for a, b, scale in jobs:
        M = 1 if a is None else a.shape[1]
        N = b.shape[1]
        assert b.stride(1) == 1 and (a is None or a.stride(1) == 1)
        o = torch.empty((M, N), dtype=torch.float32, device=dev)
        outs.append(o)
        cjobs.append(_native.LBSetJobC(None if a is None else a.data_ptr(), 0 if a is None else a.stride(0),
                                       b.data_ptr(), b.stride(0), M, N, float(scale), o.data_ptr()))
        row += M * N
    need = ((S + OS_SPAN - 1) // OS_SPAN) * row
    w = _os_work.get(dev)
    if w is None or w.numel() < need:
        w = _os_work[dev] = torch.empty(max(need, 1 << 20), dtype=torch.float32, device=dev)
    arr = (_native.LBSetJobC * len(cjobs))(*cjobs)
    _native.check(_native.lib().lb_ds_over_sets(arr, len(cjobs), S, w.data_ptr(), w.numel(), _stream(dev)))
    return outs


class _FusedDeepSetsTrain(torch.autograd.Function):
    """(x, *params) -> (logits (B, R), psi_mean (B, 64) or None).

    params: the actor's 6 equivariant weights (Lambda, Gamma per layer) followed, when a
    critic is given, by the critic psi's 6.  Gradients flow to the params only (x is data).
    """

    @staticmethod
    def forward(ctx, x, owner, actor_net, critic, *params):
        dev = x.device
        B, R, _ = x.shape
        frag = fused.packed(owner, actor_net, critic)
        logits = torch.empty((B, R), dtype=torch.float32, device=dev)
        save_a = torch.empty((2, B, R, 64), dtype=torch.float32, device=dev)
        setvec = torch.empty((B, SV), dtype=torch.float32, device=dev)
        mean = save_c = None
        if critic is not None:
            mean = torch.empty((B, 64), dtype=torch.float32, device=dev)
            save_c = torch.empty((2, B, R, 64), dtype=torch.float32, device=dev)
        _native.check(_native.lib().lb_ds_train_forward(
            frag.data_ptr(), x.data_ptr(), B, R, logits.data_ptr(), fused._ptr(mean), save_a.data_ptr(),
            fused._ptr(save_c), setvec.data_ptr(), _stream(dev)))
        ctx.actor_net, ctx.critic, ctx.owner = actor_net, critic, owner
        ctx.save_for_backward(x, save_a, save_c, setvec)
        if critic is None:
            return logits
        return logits, mean

    @staticmethod
    def backward(ctx, dlogits, dmean=None):
        x, save_a, save_c, setvec = ctx.saved_tensors
        actor_net, critic = ctx.actor_net, ctx.critic
        dev = x.device
        B, R, _ = x.shape
        if dlogits is None:
            dlogits = torch.zeros((B, R), dtype=torch.float32, device=dev)
        dlogits = dlogits.float().contiguous()
        if critic is not None:
            dmean = torch.zeros((B, 64), dtype=torch.float32, device=dev) if dmean is None else dmean.float().contiguous()
        bfrag = fused.pinned_backward(ctx.owner)  # (a DQN train period packs it with the forward's)
        if bfrag is None:
            bfrag = _pack_backward(actor_net, critic, dev)
        wgrad = torch.empty((2, _native.LB_DS_WGRAD_FLOATS), dtype=torch.float32, device=dev)
        work = _workspace(dev)
        args = (bfrag.data_ptr(), x.data_ptr(), B, R, save_a.data_ptr(), fused._ptr(save_c), dlogits.data_ptr(),
                fused._ptr(dmean), wgrad.data_ptr(), work.data_ptr(), setvec.data_ptr())
        if B <= SET_GRADS_MAX_SETS:
            # the sums over the sets with the slot reduction, in its launch (lb_ds_train_backward_sets)
            n = _native.LB_DS_SETGRAD_ACTOR + (_native.LB_DS_SETGRAD_CRITIC if critic is not None else 0)
            sg = torch.empty(n, dtype=torch.float32, device=dev)
            _native.check(_native.lib().lb_ds_train_backward_sets(*args, sg.data_ptr(), _stream(dev)))
            grads = [wgrad[0, 4096:].view(64, 8), sg[:512].view(64, 8), wgrad[0, :4096].view(64, 64),
                     sg[512:4608].view(64, 64), sg[4608:4672].view(1, 64), sg[4672:4736].view(1, 64)]
            if critic is not None:
                c = sg[_native.LB_DS_SETGRAD_ACTOR:]
                grads += [wgrad[1, 4096:].view(64, 8), c[:512].view(64, 8), wgrad[1, :4096].view(64, 64),
                          c[512:4608].view(64, 64), c[4608:8704].view(64, 64), c[8704:].view(64, 64)]
            return (None, None, None, None) + tuple(grads)
        _native.check(_native.lib().lb_ds_train_backward(*args, _stream(dev)))
        # the sums over the sets, every one in one lb_ds_over_sets call (two launches)
        max0 = _vec(setvec, "MAX0", 8)
        g3 = dlogits.sum(1, keepdim=True)
        jobs = [(_vec(setvec, "GS1A"), max0, -1.0),                            # actor Gamma1
                (_vec(setvec, "GS2A"), _vec(setvec, "MAX1A"), -1.0),           # actor Gamma2
                (None, _vec(setvec, "GA3"), 1.0),                              # actor Lambda3
                (g3, _vec(setvec, "MAX2A"), -1.0)]                             # actor Gamma3
        if critic is not None:
            jobs += [(_vec(setvec, "GS1C"), max0, -1.0),                       # critic Gamma1
                     (_vec(setvec, "GS2C"), _vec(setvec, "MAX1C"), -1.0),      # critic Gamma2
                     (dmean, _vec(setvec, "CS2"), 1.0 / R),                    # critic Lambda3
                     (dmean, _vec(setvec, "MAX2C"), -1.0)]                     # critic Gamma3
        s = sums_over_sets(jobs, B, dev)
        grads = [wgrad[0, 4096:].view(64, 8), s[0], wgrad[0, :4096].view(64, 64), s[1], s[2], s[3]]
        if critic is not None:
            grads += [wgrad[1, 4096:].view(64, 8), s[4], wgrad[1, :4096].view(64, 64), s[5], s[6], s[7]]
        return (None, None, None, None) + tuple(grads)


class _FusedQTrainWithTarget(_FusedDeepSetsTrain):
    """(x, owner, actor_net, tfrag, x_next, *params) -> (logits (B, R), q_next (B, R)): the
    actor-only training forward of _FusedDeepSetsTrain and, in the same launch
    (lb_ds_forward_pair), the Q values of x_next under the packed image tfrag (the DQN's
    target network; no gradient).  The backward is _FusedDeepSetsTrain's."""

    @staticmethod
    def forward(ctx, x, owner, actor_net, tfrag, x_next, *params):
        dev = x.device
        B, R, _ = x.shape
        frag = fused.packed(owner, actor_net, None)
        logits = torch.empty((B, R), dtype=torch.float32, device=dev)
        q_next = torch.empty((B, R), dtype=torch.float32, device=dev)
        save_a = torch.empty((2, B, R, 64), dtype=torch.float32, device=dev)
        setvec = torch.empty((B, SV), dtype=torch.float32, device=dev)
        _native.check(_native.lib().lb_ds_forward_pair(
            tfrag.data_ptr(), x_next.data_ptr(), q_next.data_ptr(), frag.data_ptr(), x.data_ptr(), logits.data_ptr(),
            save_a.data_ptr(), setvec.data_ptr(), B, R, _stream(dev)))
        ctx.actor_net, ctx.critic, ctx.owner = actor_net, None, owner
        ctx.save_for_backward(x, save_a, None, setvec)
        ctx.mark_non_differentiable(q_next)
        ctx.set_materialize_grads(False)
        return logits, q_next

    @staticmethod
    def backward(ctx, dlogits, dq_next=None):
        grads = _FusedDeepSetsTrain.backward(ctx, dlogits)
        return (None,) * 5 + tuple(grads[4:])


PAIR_MAX_ELEMENTS = 16  # lb_ds_forward_pair's sets


def q_train_with_target(owner, actor_net, x, target, x_next):
    """DQN train step forwards in one launch: (Q(x) of `owner`'s actor_net, differentiable;
    Q(x_next) of the DQNDeepSetAgent `target`, no gradient)."""
    x = x.float().contiguous()
    x_next = x_next.float().contiguous()
    tfrag = fused.packed(target, target.q_network.net, None)
    return _FusedQTrainWithTarget.apply(x, owner, actor_net, tfrag, x_next, *_eq_params(actor_net))


class _Rho(torch.autograd.Function):
    """The critic's rho = Linear(64,64) ELU Linear(64,1) on the psi means (B, 64), with the
    two weight gradients as chunked reductions over the sets (`_over_sets`): torch's Linear
    backward runs them as one K = B GEMM on one or two workgroups (120-180 us each at
    B = 51,200).  Same math as deep_sets_agent_original.py:95-97."""

    @staticmethod
    def forward(ctx, mean, w1, b1, w2, b2):
        r1 = torch.nn.functional.elu(torch.addmm(b1, mean, w1.t()))
        ctx.save_for_backward(mean, w1, w2, r1)
        return torch.addmm(b2, r1, w2.t())

    @staticmethod
    def backward(ctx, gv):
        mean, w1, w2, r1 = ctx.saved_tensors
        gv = gv.contiguous()
        gz = (gv @ w2) * torch.where(r1 > 0, torch.ones_like(r1), r1 + 1)
        S = mean.shape[0]
        if S <= SET_GRADS_MAX_SETS or not gv.is_cuda:
            return gz @ w1, _over_sets(gz, mean), gz.sum(0), _over_sets(gv, r1), gv.sum(0)
        dw1, db1, dw2, db2 = sums_over_sets([(gz, mean, 1.0), (None, gz, 1.0), (gv, r1, 1.0), (None, gv, 1.0)], S,
                                            gv.device)
        return gz @ w1, dw1, db1.view(-1), dw2, db2.view(-1)


def _eq_params(net):
    out = []
    for j in (0, 2, 4):
        out += [net[j].Lambda.weight, net[j].Gamma.weight]
    return out


def actor_critic(agent, x):
    """DeepSetAgent training forward: (logits (B, R), value (B,)), differentiable w.r.t.
    every parameter; rho runs as the agent's own torch modules on the fused psi mean."""
    actor_net, critic = agent.actor.net, agent.critic
    x = x.float().contiguous()
    logits, mean = _FusedDeepSetsTrain.apply(x, agent, actor_net, critic,
                                             *_eq_params(actor_net), *_eq_params(critic.psi))
    rho = critic.rho
    return logits, _Rho.apply(mean, rho[0].weight, rho[0].bias, rho[2].weight, rho[2].bias).squeeze(-1)


def actor_only(owner, actor_net, x):
    """EquivariantDeepSet training forward (the DQN Q network): logits (B, R)."""
    x = x.float().contiguous()
    return _FusedDeepSetsTrain.apply(x, owner, actor_net, None, *_eq_params(actor_net))


class _PPOHead(torch.autograd.Function):
    """ppo_deepset.py:227-263's loss from (logits, value) in one launch (lb_ppo_head): the
    per-set terms and the loss's gradient w.r.t. logits and value, which backward returns
    (scaled by the incoming gradient of the loss).  Returns (loss, stats) with stats =
    (pg_loss, mean value term, entropy, approx_kl, clipfrac), not differentiable."""

    @staticmethod
    def forward(ctx, logits, value, masks, actions, oldlogp, adv, ret, vold, clip, ent_coef, vf_coef, clip_vloss):
        M, R = logits.shape
        dev = logits.device
        logits = logits.float().contiguous()
        dlogits = torch.empty_like(logits)
        dvalue = torch.empty((M,), dtype=torch.float32, device=dev)
        terms = torch.empty((M, 6), dtype=torch.float32, device=dev)
        c = lambda t: t.float().contiguous()  # noqa: E731
        m = None
        if masks is not None:
            if masks.dtype != torch.bool or tuple(masks.shape) != (M, R):
                raise ValueError("masks must be (M, R) bool")
            m = masks.contiguous()
        keep = [c(actions), c(oldlogp), c(adv), c(ret), c(vold), c(value.reshape(-1))]
        _native.check(_native.lib().lb_ppo_head(
            logits.data_ptr(), fused._ptr(m), *[t.data_ptr() for t in keep], M, R, float(clip), float(ent_coef),
            float(vf_coef), int(bool(clip_vloss)), dlogits.data_ptr(), dvalue.data_ptr(), terms.data_ptr(),
            _stream(dev)))
        means = terms.mean(0)
        ctx.save_for_backward(dlogits, dvalue)
        ctx.vshape = value.shape
        stats = means[:5]
        ctx.mark_non_differentiable(stats)
        ctx.set_materialize_grads(False)  # (no zero fill for the stats' gradient)
        return means[5], stats

    @staticmethod
    def backward(ctx, gloss, gstats):
        dlogits, dvalue = ctx.saved_tensors
        if gloss is None:
            return (None,) * 12
        if is_unit_seed(gloss):  # (x * 1 == x bit for bit: no multiply launches)
            return (dlogits, dvalue.view(ctx.vshape)) + (None,) * 10
        return (dlogits * gloss, (dvalue * gloss).view(ctx.vshape)) + (None,) * 10


def ppo_head(logits, value, masks, actions, oldlogp, adv, ret, vold, clip_coef, ent_coef, vf_coef, clip_vloss):
    return _PPOHead.apply(logits, value, masks, actions, oldlogp, adv, ret, vold, clip_coef, ent_coef, vf_coef,
                          clip_vloss)


class _DQNHead(torch.autograd.Function):
    """dqn_deepset.py:180-187's loss from the trained network's Q values (lb_dqn_head): the
    TD target from the target network's Q(next_obs) (no gradient), the squared errors and
    their mean's gradient w.r.t. q, which backward returns (times the incoming gradient).
    Returns (loss, td_target, old_val); the last two are not differentiable."""

    @staticmethod
    def forward(ctx, q, q_next, actions, rewards, dones, gamma):
        M, R = q.shape
        dev = q.device
        q = q.float().contiguous()
        dq = torch.empty_like(q)
        sq = torch.empty((M,), dtype=torch.float32, device=dev)
        td = torch.empty((M,), dtype=torch.float32, device=dev)
        old = torch.empty((M,), dtype=torch.float32, device=dev)
        # (up to 1024 samples the kernel also takes the mean: no separate reduction launch)
        loss = torch.empty((), dtype=torch.float32, device=dev) if M <= DQN_HEAD_LOSS_MAX else None
        keep = [q_next.float().contiguous(), actions.reshape(-1).to(torch.int64).contiguous(),
                rewards.reshape(-1).float().contiguous(), dones.reshape(-1).float().contiguous()]
        _native.check(_native.lib().lb_dqn_head(
            q.data_ptr(), *[t.data_ptr() for t in keep], M, R, float(gamma), dq.data_ptr(), sq.data_ptr(),
            td.data_ptr(), old.data_ptr(), fused._ptr(loss), _stream(dev)))
        ctx.save_for_backward(dq)
        ctx.mark_non_differentiable(td, old)
        # (td and old get no gradient: without this autograd fills two zero tensors for them,
        # two kernels per DQN train step)
        ctx.set_materialize_grads(False)
        return (sq.mean() if loss is None else loss), td, old

    @staticmethod
    def backward(ctx, gloss, gtd, gold):
        (dq,) = ctx.saved_tensors
        if gloss is None:
            return (None,) * 6
        if is_unit_seed(gloss):  # (dq * 1 == dq bit for bit: no multiply launch)
            return dq, None, None, None, None, None
        return dq * gloss, None, None, None, None, None


DQN_HEAD_LOSS_MAX = 1024  # lb_dqn_head's one-block loss (loss_out)


def unit_seed(device, dtype=torch.float32):
    """A scalar 1 to seed loss.backward() with; the loss heads' backward recognise it (autograd
    hands the root's seed tensor itself to the head) and return their saved gradient as is
    instead of launching a multiply by 1."""
    t = torch.ones((), dtype=dtype, device=device)
    t._lbk8s_unit = True
    return t


def is_unit_seed(g):
    return getattr(g, "_lbk8s_unit", False)


def dqn_head(q, q_next, actions, rewards, dones, gamma):
    """(F.mse_loss(td, q.gather(1, actions)), td, q.gather(1, actions)) with td = rewards +
    gamma * q_next.max(1) * (1 - dones), and the loss's gradient, in one launch."""
    return _DQNHead.apply(q, q_next, actions, rewards, dones, gamma)

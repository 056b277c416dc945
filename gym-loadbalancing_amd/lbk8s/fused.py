"""Fused deep-sets forward: lb_ds_forward in liblbk8s.so.

The reference evaluates its policy with torch modules (envs/deep_sets_agent_original.py:
56-106; the DQN Q network, envs/deep_sets_agent_dqn.py:10-42).  Rollouts here call one
HIP kernel per step instead: it reads each env's (R, 8) observation once and writes the
R actor logits (or Q values) and the critic value, every layer on f32 MFMA with the
activations kept in registers (csrc/lbk8s_deepsets.h).

The kernel takes the weights in fragment order; `lb_ds_pack` builds that image from the
torch parameters on the device.  The image is cached per module and rebuilt when any
parameter's version counter moves (every optimizer step bumps it), so callers never
repack by hand.

Training runs the fused training kernels (lbk8s/fused_train.py), which use the same image.
The forward covers R <= 257 (every env the C ABI accepts: E <= 256 plus the reject row;
above 80 elements the kernel streams the set in 32-element chunks).  Inputs it does not cover (not on
a HIP device, non-reference widths) run the same torch modules on the same device;
`require=True` turns that into an error instead.
"""
import ctypes as C
import weakref

import torch

from . import _native

ENABLED = True
_cache = weakref.WeakKeyDictionary()


def _ptr(t):
    return t.data_ptr() if t is not None else None


def _weights_struct(actor_net, critic):
    w = _native.LBDSWeightsC()
    keep = []

    def put(t):
        t = t.detach().float().contiguous()
        keep.append(t)
        return t.data_ptr()

    for i, j in enumerate((0, 2, 4)):
        w.actor_lambda[i] = put(actor_net[j].Lambda.weight)
        w.actor_gamma[i] = put(actor_net[j].Gamma.weight)
    if critic is not None:
        for i, j in enumerate((0, 2, 4)):
            w.critic_lambda[i] = put(critic.psi[j].Lambda.weight)
            w.critic_gamma[i] = put(critic.psi[j].Gamma.weight)
        w.rho_w1 = put(critic.rho[0].weight)
        w.rho_b1 = put(critic.rho[0].bias)
        w.rho_w2 = put(critic.rho[2].weight)
        w.rho_b2 = put(critic.rho[2].bias)
    return w, keep


def _geometry_ok(actor_net, x):
    return (x.is_cuda and x.dim() == 3 and x.shape[-1] == 8 and 1 <= x.shape[1] <= _native.LB_DS_MAX_ELEMENTS_FWD
            and actor_net[0].Lambda.weight.shape == (64, 8) and actor_net[2].Lambda.weight.shape == (64, 64))


_pinned = weakref.WeakKeyDictionary()


def invalidate(module):
    """Drop `module`'s cached image: needed after parameter updates the version counters do
    not see (optimizer steps replayed from a HIP graph)."""
    _cache.pop(module, None)


def pin(module, frag):
    """Make `frag` (a fixed image the caller keeps current, e.g. packed at the start of a
    captured DQN train period) the image of `module` for packed(): no pack is issued, in a
    capture or not.  pin(module, None) undoes it."""
    if frag is None:
        _pinned.pop(module, None)
    else:
        _pinned[module] = frag


def packed(module, actor_net, critic):
    """Fragment image of (actor_net, critic) cached on `module`; rebuilt after any update.
    While a HIP graph is being captured the pack is always issued (and so replayed)."""
    pinned = _pinned.get(module)
    if pinned is not None:
        return pinned
    params = list(actor_net.parameters()) + (list(critic.parameters()) if critic is not None else [])
    version = tuple(p._version for p in params) + tuple(p.data_ptr() for p in params)
    hit = _cache.get(module)
    if hit is not None and hit[0] == version and not torch.cuda.is_current_stream_capturing():
        return hit[1]
    dev = params[0].device
    frag = torch.empty(_native.LB_DS_FRAG_FLOATS, dtype=torch.float32, device=dev)
    w, keep = _weights_struct(actor_net, critic)
    L = _native.lib()
    _native.check(L.lb_ds_pack(C.byref(w), frag.data_ptr(), torch.cuda.current_stream(dev).cuda_stream))
    del keep  # stream-ordered: the pack kernel is enqueued before any later reuse of the memory
    _cache[module] = (version, frag)
    return frag


def _launch(frag, x, logits, value):
    L = _native.lib()
    B, R, _ = x.shape
    _native.check(L.lb_ds_forward(frag.data_ptr(), x.data_ptr(), B, R, _ptr(logits), _ptr(value),
                                  torch.cuda.current_stream(x.device).cuda_stream))


@torch.no_grad()
def deepsets_forward(agent, x: torch.Tensor, require: bool = False):
    """(logits (B, R), value (B,)) of a DeepSetAgent, in one launch when possible."""
    actor_net = agent.actor.net
    if not (ENABLED and _geometry_ok(actor_net, x)):
        if require:
            raise RuntimeError(f"fused deep-sets forward does not cover input {tuple(x.shape)} on {x.device}")
        return agent.actor(x), agent.critic(x)
    x = x.float().contiguous()
    frag = packed(agent, actor_net, agent.critic)
    B, R, _ = x.shape
    logits = torch.empty((B, R), dtype=torch.float32, device=x.device)
    value = torch.empty((B,), dtype=torch.float32, device=x.device)
    _launch(frag, x, logits, value)
    return logits, value


@torch.no_grad()
def q_forward(qnet, x: torch.Tensor, require: bool = False):
    """Q values (B, R) of a DQNDeepSetAgent (actor-only image of its q_network)."""
    net = qnet.q_network.net
    if not (ENABLED and _geometry_ok(net, x)):
        if require:
            raise RuntimeError(f"fused deep-sets forward does not cover input {tuple(x.shape)} on {x.device}")
        return qnet.q_network(x)
    x = x.float().contiguous()
    frag = packed(qnet, net, None)
    B, R, _ = x.shape
    q = torch.empty((B, R), dtype=torch.float32, device=x.device)
    _launch(frag, x, q, None)
    return q


def frag_buffer(device):
    """A fixed weight-image buffer for q_forward_graphable."""
    return torch.empty(_native.LB_DS_FRAG_FLOATS, dtype=torch.float32, device=device)


@torch.no_grad()
def q_forward_graphable(qnet, x, out, frag):
    """Q values of a DQNDeepSetAgent into `out`, packing the live parameters into `frag`
    first: two launches on fixed buffers, so the pair can be captured in a HIP graph and
    replayed after optimizer steps (Adam updates the parameters in place)."""
    net = qnet.q_network.net
    if not _geometry_ok(net, x):
        raise RuntimeError(f"fused deep-sets forward does not cover input {tuple(x.shape)} on {x.device}")
    w, keep = _weights_struct(net, None)
    L = _native.lib()
    _native.check(L.lb_ds_pack(C.byref(w), frag.data_ptr(), torch.cuda.current_stream(x.device).cuda_stream))
    del keep
    _launch(frag, x, out, None)
    return out


def pack_q_into(qnet, frag, bfrag=None):
    """Pack a DQNDeepSetAgent's live parameters into the fixed image `frag` (one launch;
    graph-capturable: a replay re-packs the current parameters); with `bfrag`, the training
    backward's image too, in the same launch (lb_ds_pack_pair)."""
    w, keep = _weights_struct(qnet.q_network.net, None)
    stream = torch.cuda.current_stream(frag.device).cuda_stream
    if bfrag is None:
        _native.check(_native.lib().lb_ds_pack(C.byref(w), frag.data_ptr(), stream))
    else:
        _native.check(_native.lib().lb_ds_pack_pair(C.byref(w), frag.data_ptr(), bfrag.data_ptr(), stream))
    del keep
    return frag


def bwd_frag_buffer(device):
    """A fixed backward weight-image buffer (pack_q_into's bfrag)."""
    return torch.empty(_native.LB_DS_BWD_FLOATS, dtype=torch.float32, device=device)


_pinned_bwd = weakref.WeakKeyDictionary()


def pin_backward(module, bfrag):
    """As pin(), for the training backward's image of `module` (fused_train): the caller keeps
    `bfrag` current.  pin_backward(module, None) undoes it."""
    if bfrag is None:
        _pinned_bwd.pop(module, None)
    else:
        _pinned_bwd[module] = bfrag


def pinned_backward(module):
    return _pinned_bwd.get(module)


@torch.no_grad()
def q_argmax_graphable(qnet, x, masks, actions_out, frag, q_out=None):
    """Greedy actions of a DQNDeepSetAgent (dqn_deepset.py:134-142: argmax of the Q values
    with invalid actions at -1e8, first index on ties) into `actions_out` (B,) int32, in two
    launches on fixed buffers (pack into `frag`, then the forward with the argmax fused:
    lb_ds_q_argmax), so the pair can be captured in a HIP graph.  masks: (B, R) bool or None."""
    net = qnet.q_network.net
    if not _geometry_ok(net, x):
        raise RuntimeError(f"fused deep-sets forward does not cover input {tuple(x.shape)} on {x.device}")
    if masks is not None and (masks.dtype != torch.bool or tuple(masks.shape) != tuple(x.shape[:2])
                              or not masks.is_contiguous()):
        raise ValueError("masks must be a contiguous (B, R) bool tensor")
    w, keep = _weights_struct(net, None)
    L = _native.lib()
    stream = torch.cuda.current_stream(x.device).cuda_stream
    _native.check(L.lb_ds_pack(C.byref(w), frag.data_ptr(), stream))
    del keep
    B, R, _ = x.shape
    _native.check(L.lb_ds_q_argmax(frag.data_ptr(), x.data_ptr(), B, R, _ptr(masks), _ptr(q_out),
                                   actions_out.data_ptr(), stream))
    return actions_out

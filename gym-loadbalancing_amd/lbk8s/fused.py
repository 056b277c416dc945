"""Dispatch for the fused deep-sets forward (actor logits + critic value in one launch).

Until the HIP kernel lb_ds_forward is selected (lbk8s.fused.ENABLED), the two torch
modules run (on the same device as the inputs); both paths return (logits (B,R), value (B,)).
"""
import torch

ENABLED = False


def deepsets_forward(agent, x: torch.Tensor):
    return agent.actor(x), agent.critic(x)

"""A2C update restated in torch fp32 on the CPU (TEST INFRASTRUCTURE ONLY).

PARITY UNPINNED: the reference's trainer math lives in the absent deep-rl==0.2.9
(experiments/thor_cached_auxiliary.py:2-18,26-42 import it). This file states the
standard A2C the engine implements (DESIGN.md "A2C contract"), with the reference's
hyper-parameters (thor_cached_auxiliary.py:29-37):
  returns    R_T = V(s_T);  R_t = r_t + gamma * R_{t+1} * (1 - done_t)
  advantage  A_t = R_t - V(s_t)
  loss       L = value_coef * mean(A^2) - mean(A.detach() * log pi(a_t|s_t))
                 - entropy_coef * mean(H(pi(.|s_t)))
  clip       torch.nn.utils.clip_grad_norm_(params, max_norm)      (max_norm 0.5)
  optimizer  torch.optim.RMSprop(lr, alpha=0.99, eps=1e-5)         (lr 7e-4 -> 0 linear)
"""
import torch
import torch.nn.functional as F


def returns(rewards, dones, values_ext, gamma):
    """rewards, dones [T,E]; values_ext [T+1,E] (last row = bootstrap) -> returns [T,E]."""
    T = rewards.shape[0]
    R = values_ext[T].clone()
    out = torch.empty_like(rewards)
    for t in range(T - 1, -1, -1):
        R = rewards[t] + gamma * R * (1.0 - dones[t].to(rewards.dtype))
        out[t] = R
    return out


def loss(logits, values, actions, rets, value_coef=0.5, entropy_coef=0.01):
    """logits [N,A], values [N], actions [N] long, rets [N] -> (loss, stats dict)."""
    logp_all = F.log_softmax(logits, dim=-1)
    p = logp_all.exp()
    logp = logp_all.gather(1, actions.view(-1, 1)).squeeze(1)
    ent = -(p * logp_all).sum(-1)
    adv = rets - values
    value_loss = adv.pow(2).mean()
    action_loss = -(adv.detach() * logp).mean()
    entropy = ent.mean()
    total = value_coef * value_loss + action_loss - entropy_coef * entropy
    return total, dict(value_loss=value_loss, action_loss=action_loss, entropy=entropy)


def clip_and_rmsprop(params, grads, square_avg, lr, max_norm=0.5, alpha=0.99, eps=1e-5):
    """In-place on lists of tensors; returns the pre-clip total norm."""
    total = torch.sqrt(sum((g.double() ** 2).sum() for g in grads)).float()
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    for p, g, s in zip(params, grads, square_avg):
        g = g * coef
        s.mul_(alpha).addcmul_(g, g, value=1 - alpha)
        p.addcdiv_(g, s.sqrt().add_(eps), value=-lr)
    return total

"""UNREAL auxiliary losses in torch fp64 on the CPU (TEST INFRASTRUCTURE ONLY).

The checker of csrc/vn_unreal_loss.hip. The reference computes these losses in deep_rl's
UnrealTrainer (deep-rl==0.2.9, absent from the image; called from
experiments/ai2_auxiliary/trainer.py:21-43 with the weights of
experiments/thor_cached_auxiliary.py:39-41): PARITY UNPINNED. This restates the published
UNREAL algorithm as deep_rl's call sites use it (goal.py:72 pc_cell_size 4, 42 x 42 pixel
control map; thor_cached_auxiliary.py:47-48 the image observation, scaled to [0, 1]).
BigHouseModel's pixel control (models/bignet.py:77-111) has a 20 x 20 map: the same loss on
the centre 80 x 80 crop (the cell count is taken from q's shape).
"""
import torch

PC_CELLS, PC_CELL = 42, 4


def pixel_change(f0, f1, cells=PC_CELLS):
    """Pseudo-reward maps [..., cells, cells]: mean over each 4x4 cell and the 3 channels of
    |f1 - f0| / 255 on the centre crop (u8 [..., H, W, 3] frames)."""
    H, W = f0.shape[-3:-1]
    top, left = (H - cells * PC_CELL) // 2, (W - cells * PC_CELL) // 2
    crop = (slice(top, top + cells * PC_CELL), slice(left, left + cells * PC_CELL))
    d = (f1[..., crop[0], crop[1], :].double() - f0[..., crop[0], crop[1], :].double()).abs() / 255.0
    d = d.reshape(*d.shape[:-3], cells, PC_CELL, cells, PC_CELL, 3)
    return d.mean(dim=(-4, -2, -1))


def pc_loss(q, frames, actions, dones, gamma=0.9):
    """q [T+1, S, C, C, A] (C = 42, or 20 for BigHouseModel; row T: the bootstrap observation), frames u8 [T+1, S, H, W, 3],
    actions [T, S], dones [T, S] -> (mean squared TD error, d loss / d q). On a done step the
    pseudo-reward is 0: the next frame is the auto-reset frame of another episode."""
    q = q.detach().double().requires_grad_()
    T = actions.shape[0]
    C = q.shape[2]
    r = pixel_change(frames[:-1], frames[1:], C)  # [T, S, C, C]
    r = r * (~dones.bool()).double()[:, :, None, None]
    R = q[T].detach().max(-1).values
    targets = []
    for t in range(T - 1, -1, -1):
        R = r[t] + gamma * R * (~dones[t].bool()).double()[:, None, None]
        targets.append(R)
    targets = torch.stack(targets[::-1])
    qa = torch.gather(q[:T], -1, actions.long()[:, :, None, None, None].expand(-1, -1, C, C, 1))[..., 0]
    loss = ((qa - targets) ** 2).mean()
    loss.backward()
    return loss.detach(), q.grad


def rp_loss(logits, rewards, dones):
    """logits [(T-2) S, 3] of frames ts-2..ts (ts = 2..T-1, env-minor), rewards / dones [T, S]
    -> (mean cross-entropy over samples within one episode, d loss / d logits, count)."""
    T, S = rewards.shape
    logits = logits.detach().double().requires_grad_()
    ts = torch.arange(2, T).repeat_interleave(S)
    e = torch.arange(S).repeat(T - 2)
    used = ~(dones[ts - 2, e].bool() | dones[ts - 1, e].bool())
    r = rewards[ts, e]
    cls = torch.where(r == 0, 0, torch.where(r > 0, 1, 2))
    ce = torch.nn.functional.cross_entropy(logits, cls, reduction="none")
    count = int(used.sum())
    loss = (ce * used.double()).sum() / max(count, 1)
    loss.backward()
    return loss.detach(), logits.grad, count


def vr_loss(values, returns):
    """values / returns [T, S] -> (mean squared error, d loss / d values)."""
    v = values.detach().double().requires_grad_()
    loss = ((v - returns.double()) ** 2).mean()
    loss.backward()
    return loss.detach(), v.grad

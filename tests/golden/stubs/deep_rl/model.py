"""Stand-ins for deep_rl.model.{TimeDistributed, Flatten, MaskedRNN} (deep-rl 0.2.9 is not
in this image). TimeDistributed folds the leading (batch, time) dims, applies its
children in sequence and unfolds; Flatten is view(B, -1); MaskedRNN only holds its
module (its masking semantics are unknown: parity unpinned)."""
import torch.nn as nn


class TimeDistributed(nn.Sequential):
    def forward(self, x):
        b, t = x.shape[:2]
        y = super().forward(x.reshape(b * t, *x.shape[2:]))
        return y.view(b, t, *y.shape[1:])


class Flatten(nn.Module):
    def forward(self, x):
        return x.view(x.size(0), -1)


class MaskedRNN(nn.Module):
    def __init__(self, inner):
        super().__init__()
        self.inner = inner

    def forward(self, x, masks, states):
        raise NotImplementedError("MaskedRNN semantics live in deep-rl 0.2.9 (absent)")

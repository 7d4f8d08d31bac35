"""BigGoalHouseModel trunk + heads in torch fp32 on the CPU (TEST INFRASTRUCTURE ONLY).

Restates models/goal.py:36-59 and 77-92 of the reference (shared_base applied to image
and goal with shared weights, channel concat, conv_base, conv_merge Linear -> 512, ReLU,
then the policy_logits / critic Linear heads). The LSTM (goal.py:61-67) is out of the
slice: the heads read the 512-d features directly. in_features
of conv_merge is derived from the frame size (the reference hard-codes 9*9*32, valid
only for 171-178 px inputs: documented deviation). Pinned against the reference modules
by tests/golden/gen_model_goldens.py.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


def trunk_sizes(h, w):
    o1 = ((h - 7) // 4 + 1, (w - 7) // 4 + 1)
    o2 = ((o1[0] - 4) // 2 + 1, (o1[1] - 4) // 2 + 1)
    o3 = ((o2[0] - 4) // 2 + 1, (o2[1] - 4) // 2 + 1)
    return o1, o2, o3


class GoalNetOracle(nn.Module):
    def __init__(self, frame_hw=(84, 84), num_inputs=3, num_outputs=4):
        super().__init__()
        _, _, o3 = trunk_sizes(*frame_hw)
        self.conv1 = nn.Conv2d(num_inputs, 32, 7, stride=4)
        self.conv2 = nn.Conv2d(32, 32, 4, stride=2)
        self.conv3 = nn.Conv2d(64, 64, 4, stride=2)
        self.conv4 = nn.Conv2d(64, 32, 1)
        self.fc = nn.Linear(32 * o3[0] * o3[1], 512)
        self.policy_logits = nn.Linear(512, num_outputs)
        self.critic = nn.Linear(512, 1)

    def features(self, image, goal):
        """image, goal: float [N,3,H,W] (TransposeImage + ScaledFloatFrame output)."""
        def base(x):
            return F.relu(self.conv2(F.relu(self.conv1(x))))
        x = torch.cat((base(image), base(goal)), 1)
        x = F.relu(self.conv4(F.relu(self.conv3(x))))
        return F.relu(self.fc(x.flatten(1)))

    def forward(self, image, goal):
        f = self.features(image, goal)
        return self.policy_logits(f), self.critic(f)

    def forward_masked(self, image, goal, masks):
        """The same network with every ReLU replaced by multiplication with a given 0/1 mask
        (masks = dict m1i, m1g, m2i, m2g, m3, m4, m5 in NCHW / [N,512]). Fed the masks of
        the GPU forward, the gradients are those of the function the GPU differentiated,
        so a pre-activation within rounding of zero (a ReLU tie) cannot make the two
        disagree. Returns (logits, value, x4, pre) with pre = the pre-activations, for the
        check that the masks are the signs of the oracle's own pre-activations wherever
        those are not ties."""
        pre = {}

        def base(x, a, b):
            pre["z1" + a[-1]] = z1 = self.conv1(x)
            pre["z2" + a[-1]] = z2 = self.conv2(z1 * masks[a])
            return z2 * masks[b]
        x = torch.cat((base(image, "m1i", "m2i"), base(goal, "m1g", "m2g")), 1)
        pre["z3"] = z3 = self.conv3(x)
        pre["z4"] = z4 = self.conv4(z3 * masks["m3"])
        x4 = z4 * masks["m4"]
        pre["z5"] = z5 = self.fc(x4.flatten(1))
        f = z5 * masks["m5"]
        return self.policy_logits(f), self.critic(f), x4, pre

    def load_reference(self, sd):
        """Reference state-dict names (deep_rl TimeDistributed wrapping an nn.Sequential)."""
        m = {"shared_base.0.0": self.conv1, "shared_base.0.2": self.conv2,
             "conv_base.0.0": self.conv3, "conv_base.0.2": self.conv4,
             "conv_merge.0.1": self.fc, "policy_logits.0": self.policy_logits, "critic.0": self.critic}
        for k, mod in m.items():
            mod.weight.data.copy_(torch.as_tensor(sd[k + ".weight"]))
            mod.bias.data.copy_(torch.as_tensor(sd[k + ".bias"]))
        return self


class RecurrentGoalNetOracle(GoalNetOracle):
    """BigGoalHouseModel with its recurrent core: features ++ last_reward_action feed
    MaskedRNN(nn.LSTM(512 + A + 1, 512, batch_first=True)) (goal.py:61-67, 84-92) and the
    heads read the LSTM output. The LSTM cell is torch's own nn.LSTM (the reference's
    inner module). MaskedRNN lives in the absent deep-rl 0.2.9; restated here as: before
    step t, (h, c) *= masks[:, t] (0 where an episode starts) — parity unpinned for that
    convention."""

    def __init__(self, frame_hw=(84, 84), num_inputs=3, num_outputs=4):
        super().__init__(frame_hw, num_inputs, num_outputs)
        self.lstm = nn.LSTM(512 + num_outputs + 1, 512, num_layers=1, batch_first=True)

    def forward_seq(self, image, goal, last_reward_action, masks, states):
        """image, goal float [B,T,3,H,W]; last_reward_action [B,T,A+1]; masks [B,T];
        states (h, c) [B,1,512] -> (logits [B,T,A], value [B,T,1], (h, c))."""
        B, T = image.shape[:2]
        f = self.features(image.flatten(0, 1), goal.flatten(0, 1)).view(B, T, 512)
        x = torch.cat((f, last_reward_action), 2)
        h, c = states[0].transpose(0, 1), states[1].transpose(0, 1)
        outs = []
        for t in range(T):
            m = masks[:, t].reshape(1, B, 1)
            o, (h, c) = self.lstm(x[:, t:t + 1], (h * m, c * m))
            outs.append(o)
        y = torch.cat(outs, 1)
        return self.policy_logits(y), self.critic(y), (h.transpose(0, 1), c.transpose(0, 1))

    def load_reference(self, sd):
        super().load_reference(sd)
        for name in ("weight_ih_l0", "weight_hh_l0", "bias_ih_l0", "bias_hh_l0"):
            keys = [k for k in sd if k.endswith(name)]
            getattr(self.lstm, name).data.copy_(torch.as_tensor(sd[keys[0]]))
        return self


class AuxHeadsOracle(nn.Module):
    """AuxiliaryBigGoalHouseModel's deconv heads (models/goal.py:144-189): from the
    conv_base features [N,32,h3,w3], three TimeDistributed(ConvTranspose2d(32,16,4,2), ReLU,
    ConvTranspose2d(16,C,4,2)) heads for depth (C=1), segmentation (3) and goal
    segmentation (3). Init as init_weights (goal.py:26-30: bias 0, U(+-1/sqrt(fan_in)))."""

    def __init__(self):
        super().__init__()
        self.heads = nn.ModuleList()
        for c in (1, 3, 3):
            self.heads.append(nn.Sequential(nn.ConvTranspose2d(32, 16, 4, stride=2), nn.ReLU(),
                                            nn.ConvTranspose2d(16, c, 4, stride=2)))

    def forward(self, features):
        return tuple(h(features) for h in self.heads)

    def forward_masked(self, features, masks):
        """forward() with each head's ReLU replaced by its given 0/1 mask [N,16,AH,AW]
        (see GoalNetOracle.forward_masked); returns (predictions, pre-activations)."""
        pre = [h[0](features) for h in self.heads]
        return tuple(h[2](z * m) for h, z, m in zip(self.heads, pre, masks)), pre

    def load_reference(self, sd):
        for h, name in zip(self.heads, ("deconv_depth", "deconv_mask", "deconv_mask_goal")):
            for i, layer in ((1, h[0]), (3, h[2])):
                layer.weight.data.copy_(torch.as_tensor(sd["%s.0.%d.weight" % (name, i)]))
                layer.bias.data.copy_(torch.as_tensor(sd["%s.0.%d.bias" % (name, i)]))
        return self


def autocrop(x, cell, output_size):
    """Centre crop of [..., H, W] to output_size * cell (restatement of deep_rl's
    autocrop_observations as called at experiments/ai2_auxiliary/trainer.py:11; deep-rl is
    absent, so the centring convention is parity unpinned)."""
    H, W = x.shape[-2:]
    nh, nw = output_size[0] * cell, output_size[1] * cell
    top, left = (H - nh) // 2, (W - nw) // 2
    return x[..., top:top + nh, left:left + nw]


def aux_targets(depth_u8, seg_u8, goal_seg_u8, cell, output_size):
    """compute_auxiliary_target (experiments/ai2_auxiliary/trainer.py:9-15) for the three
    aux observations (uint8 [N,H,W,C], scaled by 1/255 as the float observation wrappers
    do): autocrop, then avg_pool2d(cell, stride=cell) -> [N,C,oh,ow]."""
    out = []
    for x in (depth_u8, seg_u8, goal_seg_u8):
        t = torch.as_tensor(x).permute(0, 3, 1, 2).to(torch.float32) / 255.0
        out.append(F.avg_pool2d(autocrop(t, cell, output_size), cell, stride=cell))
    return tuple(out)


def aux_loss(predictions, targets):
    """_deconv_loss (experiments/ai2_auxiliary/trainer.py:45-55): sum of per-head MSE."""
    return sum(F.mse_loss(p, t) for p, t in zip(predictions, targets))


class BigHouseOracle(nn.Module):
    """BigHouseModel (models/bignet.py:26-75): conv_base Conv(3,32,k8,s4) ReLU, Conv(32,64,k4,s2)
    ReLU, Conv(64,32,k3) ReLU; conv_merge Linear(7*7*32, 512) ReLU; heads; the recurrent core
    as RecurrentGoalNetOracle (MaskedRNN convention unpinned). Image only."""

    def __init__(self, num_outputs=4):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 32, 8, stride=4)
        self.conv2 = nn.Conv2d(32, 64, 4, stride=2)
        self.conv3 = nn.Conv2d(64, 32, 3)
        self.fc = nn.Linear(7 * 7 * 32, 512)
        self.policy_logits = nn.Linear(512, num_outputs)
        self.critic = nn.Linear(512, 1)
        self.lstm = nn.LSTM(512 + num_outputs + 1, 512, num_layers=1, batch_first=True)

    def features(self, image):
        x = F.relu(self.conv3(F.relu(self.conv2(F.relu(self.conv1(image))))))
        return F.relu(self.fc(x.flatten(1)))

    def forward(self, image):
        f = self.features(image)
        return self.policy_logits(f), self.critic(f)

    def forward_seq(self, image, last_reward_action, masks, states):
        B, T = image.shape[:2]
        x = torch.cat((self.features(image.flatten(0, 1)).view(B, T, 512), last_reward_action), 2)
        h, c = states[0].transpose(0, 1), states[1].transpose(0, 1)
        outs = []
        for t in range(T):
            m = masks[:, t].reshape(1, B, 1)
            o, (h, c) = self.lstm(x[:, t:t + 1], (h * m, c * m))
            outs.append(o)
        y = torch.cat(outs, 1)
        return self.policy_logits(y), self.critic(y), (h.transpose(0, 1), c.transpose(0, 1))

    def load_reference(self, sd):
        m = {"conv_base.0.0": self.conv1, "conv_base.0.2": self.conv2, "conv_base.0.4": self.conv3,
             "conv_merge.0.1": self.fc, "policy_logits.0": self.policy_logits, "critic.0": self.critic}
        for k, mod in m.items():
            mod.weight.data.copy_(torch.as_tensor(sd[k + ".weight"]))
            mod.bias.data.copy_(torch.as_tensor(sd[k + ".bias"]))
        for name in ("weight_ih_l0", "weight_hh_l0", "bias_ih_l0", "bias_hh_l0"):
            keys = [k for k in sd if k.endswith(name)]
            if keys:
                getattr(self.lstm, name).data.copy_(torch.as_tensor(sd[keys[0]]))
        return self


BIGHOUSE_PARAM_ORDER = (  # BigHouseModel.named_parameters() order for the trunk + heads
    "conv_base.0.0.weight", "conv_base.0.0.bias", "conv_base.0.2.weight", "conv_base.0.2.bias",
    "conv_base.0.4.weight", "conv_base.0.4.bias", "conv_merge.0.1.weight", "conv_merge.0.1.bias",
    "critic.0.weight", "critic.0.bias", "policy_logits.0.weight", "policy_logits.0.bias",
)
BIGHOUSE_SHAPES = {
    "conv_base.0.0.weight": (32, 3, 8, 8), "conv_base.0.0.bias": (32,),
    "conv_base.0.2.weight": (64, 32, 4, 4), "conv_base.0.2.bias": (64,),
    "conv_base.0.4.weight": (32, 64, 3, 3), "conv_base.0.4.bias": (32,),
    "conv_merge.0.1.weight": (512, 1568), "conv_merge.0.1.bias": (512,),
    "critic.0.weight": (1, 512), "critic.0.bias": (1,),
    "policy_logits.0.weight": (4, 512), "policy_logits.0.bias": (4,),
}


def seeded_bighouse_state(seed):
    """tests/golden/gen_model_goldens.py:seeded_weights over BigHouseModel's trunk + heads."""
    import numpy as np
    rng = np.random.default_rng(seed)
    out = {}
    for name in BIGHOUSE_PARAM_ORDER:
        shape = BIGHOUSE_SHAPES[name]
        if name.endswith("bias"):
            v = rng.uniform(-0.05, 0.05, size=shape)
        else:
            d = 1.0 / np.sqrt(int(np.prod(shape[1:])))
            v = rng.uniform(-d, d, size=shape)
        out[name] = v.astype(np.float32)
    return out


def frames_to_float(u8):
    """uint8 [...,H,W,C] -> float32 [...,C,H,W] / 255 (TransposeImage + ScaledFloatFrame)."""
    x = torch.as_tensor(u8)
    return x.permute(*range(x.dim() - 3), -1, -3, -2).to(torch.float32) / 255.0


REFERENCE_PARAM_ORDER = (  # BigGoalHouseModel.named_parameters() order for the used modules
    "shared_base.0.0.weight", "shared_base.0.0.bias", "shared_base.0.2.weight", "shared_base.0.2.bias",
    "conv_base.0.0.weight", "conv_base.0.0.bias", "conv_base.0.2.weight", "conv_base.0.2.bias",
    "conv_merge.0.1.weight", "conv_merge.0.1.bias", "critic.0.weight", "critic.0.bias",
    "policy_logits.0.weight", "policy_logits.0.bias",
)


AUX_PARAM_ORDER = tuple("%s.0.%d.%s" % (h, i, k) for h in ("deconv_depth", "deconv_mask", "deconv_mask_goal")
                        for i in (1, 3) for k in ("weight", "bias"))


def reference_shapes(frame_hw=(84, 84), num_outputs=4):
    _, _, o3 = trunk_sizes(*frame_hw)
    aux = {}
    for h, c in (("deconv_depth", 1), ("deconv_mask", 3), ("deconv_mask_goal", 3)):
        aux.update({h + ".0.1.weight": (32, 16, 4, 4), h + ".0.1.bias": (16,),
                    h + ".0.3.weight": (16, c, 4, 4), h + ".0.3.bias": (c,)})
    return {**aux,
        "shared_base.0.0.weight": (32, 3, 7, 7), "shared_base.0.0.bias": (32,),
        "shared_base.0.2.weight": (32, 32, 4, 4), "shared_base.0.2.bias": (32,),
        "conv_base.0.0.weight": (64, 64, 4, 4), "conv_base.0.0.bias": (64,),
        "conv_base.0.2.weight": (32, 64, 1, 1), "conv_base.0.2.bias": (32,),
        "conv_merge.0.1.weight": (512, 32 * o3[0] * o3[1]), "conv_merge.0.1.bias": (512,),
        "critic.0.weight": (1, 512), "critic.0.bias": (1,),
        "policy_logits.0.weight": (num_outputs, 512), "policy_logits.0.bias": (num_outputs,),
    }


def seeded_reference_state(frame_hw, seed, aux=False):
    """The weights tests/golden/gen_model_goldens.py:seeded_weights draws (PCG64); aux adds
    the deconv heads (drawn after the trunk and heads, named_parameters order)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    shapes = reference_shapes(frame_hw)
    out = {}
    for name in REFERENCE_PARAM_ORDER + (AUX_PARAM_ORDER if aux else ()):
        shape = shapes[name]
        if name.endswith("bias"):
            v = rng.uniform(-0.05, 0.05, size=shape)
        else:
            d = 1.0 / np.sqrt(int(np.prod(shape[1:])))
            v = rng.uniform(-d, d, size=shape)
        out[name] = v.astype(np.float32)
    return out


UNREAL_PARAM_ORDER = (  # BigGoalHouseModel.named_parameters() order of pc_base, pc_action, pc_value, rp
    "pc_base.0.0.weight", "pc_base.0.0.bias", "pc_action.0.0.weight", "pc_action.0.0.bias",
    "pc_action.0.2.weight", "pc_action.0.2.bias", "pc_value.0.0.weight", "pc_value.0.0.bias",
    "pc_value.0.2.weight", "pc_value.0.2.bias", "rp.1.weight", "rp.1.bias",
)


def unreal_shapes(frame_hw=(174, 174), num_outputs=4):
    """goal.py:94-119; rp's in_features derived from the frame (the reference fixes 9*9*32*3,
    the 174x174 value)."""
    _, _, o3 = trunk_sizes(*frame_hw)
    return {"pc_base.0.0.weight": (32 * 9 * 9, 512), "pc_base.0.0.bias": (32 * 9 * 9,),
            "pc_action.0.0.weight": (32, 32, 4, 4), "pc_action.0.0.bias": (32,),
            "pc_action.0.2.weight": (32, 1, 4, 4), "pc_action.0.2.bias": (1,),
            "pc_value.0.0.weight": (32, 32, 4, 4), "pc_value.0.0.bias": (32,),
            "pc_value.0.2.weight": (32, num_outputs, 4, 4), "pc_value.0.2.bias": (num_outputs,),
            "rp.1.weight": (3, 3 * 32 * o3[0] * o3[1]), "rp.1.bias": (3,)}


def seeded_unreal_state(frame_hw, seed, num_outputs=4):
    """gen_model_goldens.py:seeded_weights over the four UNREAL modules alone (PCG64)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    shapes = unreal_shapes(frame_hw, num_outputs)
    out = {}
    for name in UNREAL_PARAM_ORDER:
        shape = shapes[name]
        if name.endswith("bias"):
            v = rng.uniform(-0.05, 0.05, size=shape)
        else:
            d = 1.0 / np.sqrt(int(np.prod(shape[1:])))
            v = rng.uniform(-d, d, size=shape)
        out[name] = v.astype(np.float32)
    return out


def pixel_control(sd, h, masks=None):
    """goal.py:131-137 after _forward_base: q [N, A, 42, 42] of features h [N, 512], in the
    dtype of h (float64 for the parity tests); sd tensors in that dtype. masks (optional):
    the ReLU masks of a run under test ({"pc_base": [N, 32, 9, 9], "pc_value.0" / "pc_action.0"
    [N, 32, 20, 20], "pc_value.2" [N, A, 42, 42], "pc_action.2" [N, 1, 42, 42]}) replace the
    oracle's own, so a pre-activation within rounding of zero cannot flip a mask between them."""
    def act(x, key):
        return F.relu(x) if masks is None else x * masks[key].to(x.dtype)

    f = act(F.linear(h, sd["pc_base.0.0.weight"], sd["pc_base.0.0.bias"]).view(-1, 32, 9, 9), "pc_base")

    def branch(name):
        x = act(F.conv_transpose2d(f, sd[name + ".0.0.weight"], sd[name + ".0.0.bias"], stride=2), name + ".0")
        return act(F.conv_transpose2d(x, sd[name + ".0.2.weight"], sd[name + ".0.2.bias"], stride=2), name + ".2")

    a = branch("pc_action")
    return branch("pc_value") + a - a.mean(1, keepdim=True)


def reward_prediction(sd, feats):
    """goal.py:121-129 after conv_base: logits [R, 3] of feats [R, 3, 32, h3, w3] (Flatten =
    view(R, -1))."""
    return F.linear(feats.reshape(feats.shape[0], -1), sd["rp.1.weight"], sd["rp.1.bias"])


BIGHOUSE_UNREAL_PARAM_ORDER = (  # BigHouseModel.named_parameters() order of pc_base, pc_action, pc_value, rp
    "pc_base.0.0.weight", "pc_base.0.0.bias", "pc_action.0.0.weight", "pc_action.0.0.bias",
    "pc_value.0.0.weight", "pc_value.0.0.bias", "rp.weight", "rp.bias",
)


def bighouse_unreal_shapes(num_outputs=4, fcin=7 * 7 * 32):
    """bignet.py:77-96: pc_base Linear(512, 32*9*9), pc_action ConvTranspose2d(32, 1, 4, 2),
    pc_value ConvTranspose2d(32, A, 4, 2); rp Linear(3 * fcin, 3) (bignet.py:96 writes 9*9*32*3,
    which fits only 100x100 frames: at 84x84 conv_base ends at 7x7, in_features derived)."""
    return {"pc_base.0.0.weight": (32 * 9 * 9, 512), "pc_base.0.0.bias": (32 * 9 * 9,),
            "pc_action.0.0.weight": (32, 1, 4, 4), "pc_action.0.0.bias": (1,),
            "pc_value.0.0.weight": (32, num_outputs, 4, 4), "pc_value.0.0.bias": (num_outputs,),
            "rp.weight": (3, 3 * fcin), "rp.bias": (3,)}


def seeded_bighouse_unreal_state(seed, num_outputs=4):
    """gen_model_goldens.py:seeded_weights over BigHouseModel's four UNREAL modules (PCG64)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    shapes = bighouse_unreal_shapes(num_outputs)
    out = {}
    for name in BIGHOUSE_UNREAL_PARAM_ORDER:
        shape = shapes[name]
        if name.endswith("bias"):
            v = rng.uniform(-0.05, 0.05, size=shape)
        else:
            d = 1.0 / np.sqrt(int(np.prod(shape[1:])))
            v = rng.uniform(-d, d, size=shape)
        out[name] = v.astype(np.float32)
    return out


def bighouse_pixel_control(sd, h, masks=None):
    """bignet.py:105-111 after _forward_base: q [N, A, 20, 20] of features h [N, 512]: pc_base
    (Linear + ReLU) viewed (32, 9, 9), one ConvTranspose2d(k4, s2) + ReLU per branch, value +
    action - mean(action). masks (optional): the ReLU masks of a run under test ({"pc_base"
    [N, 32, 9, 9], "pc_value" [N, A, 20, 20], "pc_action" [N, 1, 20, 20]})."""
    def act(x, key):
        return F.relu(x) if masks is None else x * masks[key].to(x.dtype)

    f = act(F.linear(h, sd["pc_base.0.0.weight"], sd["pc_base.0.0.bias"]).view(-1, 32, 9, 9), "pc_base")
    a = act(F.conv_transpose2d(f, sd["pc_action.0.0.weight"], sd["pc_action.0.0.bias"], stride=2), "pc_action")
    v = act(F.conv_transpose2d(f, sd["pc_value.0.0.weight"], sd["pc_value.0.0.bias"], stride=2), "pc_value")
    return v + a - a.mean(1, keepdim=True)


def bighouse_reward_prediction(sd, feats):
    """bignet.py:98-103 after conv_base: logits [R, 3] of feats [R, 3, 32, h3, w3]."""
    return F.linear(feats.reshape(feats.shape[0], -1), sd["rp.weight"], sd["rp.bias"])

"""The goal-conditioned CNN policy on libvnav.so's MFMA kernels.

GoalNavPolicy mirrors BigGoalHouseModel's interface (models/goal.py:15-92):
``forward(inputs, masks, states) -> [policy_logits, critic, states]`` and
``initial_states(batch)``, with the trunk + heads (goal.py:36-59) computed by the HIP
kernels. ``recurrent=True`` adds the recurrent core MaskedRNN(nn.LSTM(512 + A + 1, 512))
(goal.py:61-67, 91-92): conv_merge features concatenated with the last (one-hot action,
reward) feed the LSTM, whose output feeds the heads, and ``states`` = (h, c) [B,1,512]
are carried; masks [B,T] zero the carried state where an episode starts. Without it the
features feed the heads directly and ``states`` pass through (the feed-forward slice).

All parameters live in ONE flat fp32 device buffer (layout in include/vnav.h), so the
optimizer, the gradient norm and the RCCL all-reduce each touch one contiguous tensor.
"""
import ctypes
import math
import re
import warnings

import numpy as np
import torch

from . import _lib

LAYERS = ("conv1", "conv2", "conv3", "conv4", "fc", "head")
OUT_LD = 8
PC_MAP, PC_A1, PC_P = 9, 20, 42  # pixel-control maps (goal.py:96-112)
PC_BASE = 32 * PC_MAP * PC_MAP



class Frames(ctypes.Structure):
    """vn_frames (include/vnav.h)."""
    _fields_ = [("image", ctypes.c_void_p), ("goal", ctypes.c_void_p), ("image_rows", ctypes.c_void_p),
                ("goal_rows", ctypes.c_void_p), ("frame_bytes", ctypes.c_int64), ("image_f32", ctypes.c_void_p),
                ("goal_f32", ctypes.c_void_p)]


def frames_from_batch(image, goal):
    """Dense frames: uint8 [n,H,W,3] (env output) or float [n,3,H,W] (reference wrappers)."""
    f = Frames()
    if image.dtype == torch.uint8:
        f.image, f.goal = image.data_ptr(), goal.data_ptr()
        f.frame_bytes = int(np.prod(image.shape[1:]))
    else:
        f.image_f32, f.goal_f32 = image.data_ptr(), goal.data_ptr()
    return f


def frames_from_rows(arena_ptr, frame_bytes, img_rows, goal_rows):
    """Zero-copy frames: rows of the VectorEnv scene-cache arena."""
    f = Frames()
    f.image = f.goal = arena_ptr
    f.image_rows, f.goal_rows = img_rows.data_ptr(), goal_rows.data_ptr()
    f.frame_bytes = frame_bytes
    return f


def trunk_sizes(h, w):
    o1 = ((h - 7) // 4 + 1, (w - 7) // 4 + 1)
    o2 = ((o1[0] - 4) // 2 + 1, (o1[1] - 4) // 2 + 1)
    o3 = ((o2[0] - 4) // 2 + 1, (o2[1] - 4) // 2 + 1)
    return o1, o2, o3


class AuxTargets(ctypes.Structure):
    """vn_aux_targets (include/vnav.h)."""
    _fields_ = [("table", ctypes.c_void_p), ("image_rows", ctypes.c_void_p), ("goal_rows", ctypes.c_void_p)]


AUX_HEADS = (("deconv_depth", 1, 0), ("deconv_mask", 3, 1), ("deconv_mask_goal", 3, 4))  # name, C, first out ch


class PolicyNet:
    """Handle on a vn_policy: flat parameter layout, forward/backward launches."""

    def __init__(self, frame_hw=(84, 84), num_actions=4, device=None, recurrent=False, aux=False, arch="goal",
                 unreal=False):
        """arch "goal": BigGoalHouseModel (models/goal.py); "bighouse": BigHouseModel
        (models/bignet.py, image only, 84x84). unreal: BigGoalHouseModel's pixel-control and
        reward-prediction heads (goal.py:94-133, VN_POLICY_UNREAL)."""
        self.lib = _lib.load()
        if arch not in ("goal", "bighouse"):
            raise ValueError("arch must be 'goal' or 'bighouse'")
        self.arch = arch
        self.recurrent = bool(recurrent)
        self.aux = bool(aux)
        self.unreal = bool(unreal)
        self.frame_hw = tuple(frame_hw)
        self.num_actions = int(num_actions)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else
                                   torch.device(device).index or 0)
        h = ctypes.c_void_p()
        # VN_POLICY_LSTM | VN_POLICY_AUX | VN_POLICY_BIGHOUSE
        flags = (1 if recurrent else 0) | (2 if aux else 0) | (4 if arch == "bighouse" else 0) | (8 if unreal else 0)
        with torch.cuda.device(self.device):  # the policy's split-K scratch lives on its device
            _lib.check(self.lib.vn_policy_create_ex(frame_hw[0], frame_hw[1], num_actions, flags, ctypes.byref(h)),
                       "vn_policy_create_ex")
        self._h = h
        n, a = ctypes.c_int64(), ctypes.c_int64()
        lay = (ctypes.c_int64 * 12)()
        _lib.check(self.lib.vn_policy_info(h, ctypes.byref(n), ctypes.byref(a), lay), "vn_policy_info")
        self.n_params = n.value
        self.act_floats = a.value
        self.offsets = {name: (lay[2 * i], lay[2 * i + 1]) for i, name in enumerate(LAYERS)}
        if arch == "bighouse":
            self.o3 = (7, 7)
            self.fc_in = 32 * 7 * 7
            self.shapes = {"conv1": (32, 192), "conv2": (64, 512), "conv3": (32, 576), "conv4": (0, 0),
                           "fc": (512, self.fc_in), "head": (num_actions + 1, 512)}
            self.fan_in = {"conv1": 192, "conv2": 512, "conv3": 576, "conv4": 1, "fc": self.fc_in, "head": 512}
        else:
            _, _, self.o3 = trunk_sizes(*frame_hw)
            self.fc_in = 32 * self.o3[0] * self.o3[1]
            self.shapes = {"conv1": (32, 148), "conv2": (32, 512), "conv3": (64, 1024), "conv4": (32, 64),
                           "fc": (512, self.fc_in), "head": (num_actions + 1, 512)}
            self.fan_in = {"conv1": 147, "conv2": 512, "conv3": 1024, "conv4": 64, "fc": self.fc_in, "head": 512}
        self.lstm = None
        if self.recurrent:
            info = (ctypes.c_int64 * 8)()
            _lib.check(self.lib.vn_policy_lstm_info(h, info), "vn_policy_lstm_info")
            self.lstm = dict(w=info[0], bih=info[1], bhh=info[2], xcat=info[3], xoff=info[4], lin=info[5],
                             hidden=info[6])
        self.aux_layout = None
        if self.aux:
            info = (ctypes.c_int64 * 8)()
            _lib.check(self.lib.vn_policy_aux_info(h, info), "vn_policy_aux_info")
            self.aux_layout = dict(w1=info[0], b1=info[1], w2=info[2], b2=info[3], a_hw=(info[4], info[5]),
                                   p_hw=(info[6], info[7]))
        self.unreal_layout = None
        # pixel-control map side and first deconv width: BigGoalHouseModel's two k4 s2 layers
        # (32 -> 64 -> 8, 42x42), BigHouseModel's one (32 -> 8, 20x20; bignet.py:77-91)
        self.pc_side, self.pc_c1 = (PC_A1, 8) if arch == "bighouse" else (PC_P, 64)
        if self.unreal:
            info = (ctypes.c_int64 * 8)()
            _lib.check(self.lib.vn_policy_unreal_info(h, info), "vn_policy_unreal_info")
            self.unreal_layout = dict(zip(("pc_w", "pc_b", "w1", "b1", "w2", "b2", "rp_w", "rp_b"), info[:8]))

    def check_frames(self, image, goal):
        """Dense frame batches are read by the kernels through raw pointers at this net's
        geometry: refuse any other shape, dtype, device or layout before a launch."""
        H, W = self.frame_hw
        for name, t in (("image", image), ("goal", goal)):
            if not isinstance(t, torch.Tensor) or t.device != self.device or not t.is_contiguous():
                raise ValueError("%s frames must be a contiguous tensor on %s" % (name, self.device))
            want = {torch.uint8: (H, W, 3), torch.float32: (3, H, W)}.get(t.dtype)
            if want is None or t.dim() != 4 or tuple(t.shape[1:]) != want:
                raise ValueError("%s frames must be uint8 [n,%d,%d,3] or float32 [n,3,%d,%d] (got %s %s)"
                                 % (name, H, W, H, W, t.dtype, tuple(t.shape)))
        if image.dtype != goal.dtype or image.shape[0] != goal.shape[0]:
            raise ValueError("image and goal frames must have the same dtype and batch size")

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                self.lib.vn_policy_destroy(self._h)
                self._h = None
        except Exception:
            pass

    # -- parameter layout -----------------------------------------------------------
    def views(self, flat):
        """{layer: (W [Cout][K], b [Cout])} views into a flat buffer."""
        out = {}
        for name in LAYERS:
            w, b = self.offsets[name]
            co, k = self.shapes[name]
            out[name] = (flat[w:w + co * k].view(co, k), flat[b:b + co])
        if self.lstm:
            L = self.lstm
            out["lstm"] = (flat[L["w"]:L["w"] + 2048 * L["xcat"]].view(2048, L["xcat"]),
                           flat[L["bih"]:L["bih"] + 2048], flat[L["bhh"]:L["bhh"] + 2048])
        if self.aux_layout:
            X = self.aux_layout
            out["aux"] = (flat[X["w1"]:X["w1"] + 32 * 16 * 48].view(32, 4, 4, 48), flat[X["b1"]:X["b1"] + 48],
                          flat[X["w2"]:X["w2"] + 48 * 16 * 8].view(48, 4, 4, 8), flat[X["b2"]:X["b2"] + 8])
        if self.unreal_layout:
            U = self.unreal_layout
            k, c1 = 3 * self.fc_in, self.pc_c1
            out["unreal"] = dict(
                pc_w=flat[U["pc_w"]:U["pc_w"] + PC_BASE * 512].view(PC_BASE, 512), pc_b=flat[U["pc_b"]:U["pc_b"] + PC_BASE],
                w1=flat[U["w1"]:U["w1"] + 32 * 16 * c1].view(32, 4, 4, c1), b1=flat[U["b1"]:U["b1"] + c1],
                rp_w=flat[U["rp_w"]:U["rp_w"] + 3 * k].view(3, k), rp_b=flat[U["rp_b"]:U["rp_b"] + 4])
            if self.arch == "goal":
                out["unreal"].update(w2=flat[U["w2"]:U["w2"] + 64 * 16 * 8].view(64, 4, 4, 8), b2=flat[U["b2"]:U["b2"] + 8])
        return out

    def new_params(self):
        return torch.zeros(self.n_params, dtype=torch.float32, device=self.device)

    def init_params(self, seed=0):
        """init_weights (goal.py:26-30, bignet.py:17-21): bias 0, W ~ U(+-1/sqrt(fan_in))."""
        g = torch.Generator(device="cpu").manual_seed(seed)
        flat = torch.zeros(self.n_params, dtype=torch.float32)
        v = self.views(flat)
        for name in LAYERS:
            w, _ = v[name]
            if w.numel() == 0:
                continue
            d = 1.0 / math.sqrt(self.fan_in[name])
            k = 147 if (name == "conv1" and self.arch == "goal") else w.shape[1]
            w[:, :k].uniform_(-d, d, generator=g)
        if self.lstm:  # goal.py:17-24: xavier_uniform W_ih, orthogonal W_hh, zero biases
            L = self.lstm
            wcat, _, _ = v["lstm"]
            wih = torch.empty(2048, L["lin"])
            torch.nn.init.xavier_uniform_(wih, generator=g)
            whh = torch.empty(2048, 512)
            torch.nn.init.orthogonal_(whh, generator=g)
            wcat[:, :L["lin"]] = wih
            wcat[:, L["xoff"]:] = whh
        if self.aux_layout:  # init_weights on ConvTranspose2d: fan_in = out_channels * k * k (torch's convention)
            w1, _, w2, _ = v["aux"]
            for hd, (_, c, o) in enumerate(AUX_HEADS):
                d1, d2 = 1.0 / math.sqrt(16 * 16), 1.0 / math.sqrt(c * 16)
                w1[:, :, :, 16 * hd:16 * hd + 16].uniform_(-d1, d1, generator=g)
                w2[16 * hd:16 * hd + 16, :, :, o:o + c].uniform_(-d2, d2, generator=g)
        if self.unreal_layout:  # goal.py:26-30 (bignet.py:17-21) on pc_base, the ConvTranspose2d and rp
            u, A = v["unreal"], self.num_actions
            d = 1.0 / math.sqrt(512)
            u["pc_w"].uniform_(-d, d, generator=g)
            # ConvTranspose2d's fan_in = out_channels x 16 (torch's convention)
            dv = 1.0 / math.sqrt(16 * A)
            if self.arch == "bighouse":
                u["w1"][..., :A].uniform_(-dv, dv, generator=g)
                u["w1"][..., A].uniform_(-0.25, 0.25, generator=g)
            else:
                u["w1"].uniform_(-d, d, generator=g)  # 32 out channels x 16
                u["w2"][:32, :, :, :A].uniform_(-dv, dv, generator=g)
                u["w2"][32:, :, :, A].uniform_(-0.25, 0.25, generator=g)
            d = 1.0 / math.sqrt(u["rp_w"].shape[1])
            u["rp_w"].uniform_(-d, d, generator=g)
        return flat.to(self.device)

    def from_reference(self, sd, init=None):
        """Reference state dict (BigGoalHouseModel names, any prefix) -> flat params. ``init``
        (flat params) supplies what the state dict cannot: BigHouseModel's rp weight as the
        reference builds it, Linear(9*9*32*3, 3) (bignet.py:94), fits only 100x100 frames; on
        other frames it is left at ``init`` (zeros without one) with a warning."""
        flat = torch.zeros(self.n_params, dtype=torch.float32) if init is None else \
            init.detach().float().cpu().clone()
        v = self.views(flat)
        pick = _ReferenceNames(sd)
        t = lambda x: torch.as_tensor(np.asarray(x), dtype=torch.float32)  # noqa: E731
        o3 = self.o3
        if self.arch == "bighouse":  # bignet.py:28-41: conv_base = Conv k8s4, k4s2, k3; conv_merge Linear
            for i, (name, k, co) in enumerate((("conv1", 192, 32), ("conv2", 512, 64), ("conv3", 576, 32))):
                w, b = v[name]
                w[:] = t(pick("conv_base", i, "weight")).permute(0, 2, 3, 1).reshape(co, k)
                b[:] = t(pick("conv_base", i, "bias"))
        else:
            w, b = v["conv1"]
            w[:, :147] = t(pick("shared_base", 0, "weight")).permute(0, 2, 3, 1).reshape(32, 147)
            b[:] = t(pick("shared_base", 0, "bias"))
            w, b = v["conv2"]
            w[:] = t(pick("shared_base", 1, "weight")).permute(0, 2, 3, 1).reshape(32, 512)
            b[:] = t(pick("shared_base", 1, "bias"))
            w, b = v["conv3"]
            w[:] = t(pick("conv_base", 0, "weight")).permute(0, 2, 3, 1).reshape(64, 1024)
            b[:] = t(pick("conv_base", 0, "bias"))
            w, b = v["conv4"]
            w[:] = t(pick("conv_base", 1, "weight")).reshape(32, 64)
            b[:] = t(pick("conv_base", 1, "bias"))
        w, b = v["fc"]
        w[:] = t(pick("conv_merge", 0, "weight")).view(512, 32, o3[0], o3[1]).permute(0, 2, 3, 1).reshape(512, -1)
        b[:] = t(pick("conv_merge", 0, "bias"))
        w, b = v["head"]
        A = self.num_actions
        w[:A] = t(pick("policy_logits", 0, "weight"))
        b[:A] = t(pick("policy_logits", 0, "bias"))
        w[A] = t(pick("critic", 0, "weight")).view(-1)
        b[A] = t(pick("critic", 0, "bias")).view(())
        if self.lstm:
            L = self.lstm
            wcat, bih, bhh = v["lstm"]
            wcat[:, :L["lin"]] = t(_lstm_param(sd, "weight_ih_l0"))
            wcat[:, L["xoff"]:] = t(_lstm_param(sd, "weight_hh_l0"))
            bih[:] = t(_lstm_param(sd, "bias_ih_l0"))
            bhh[:] = t(_lstm_param(sd, "bias_hh_l0"))
        if self.aux_layout:
            w1, b1, w2, b2 = v["aux"]
            for hd, (name, c, o) in enumerate(AUX_HEADS):
                w1[:, :, :, 16 * hd:16 * hd + 16] = t(sd["%s.0.1.weight" % name]).permute(0, 2, 3, 1)
                b1[16 * hd:16 * hd + 16] = t(sd["%s.0.1.bias" % name])
                w2[16 * hd:16 * hd + 16, :, :, o:o + c] = t(sd["%s.0.3.weight" % name]).permute(0, 2, 3, 1)
                b2[o:o + c] = t(sd["%s.0.3.bias" % name])
        if self.unreal_layout:
            u, A, m = v["unreal"], self.num_actions, PC_MAP
            u["pc_w"][:] = t(pick("pc_base", 0, "weight")).view(32, m, m, 512).permute(1, 2, 0, 3).reshape(PC_BASE, 512)
            u["pc_b"][:] = t(pick("pc_base", 0, "bias")).view(32, m, m).permute(1, 2, 0).reshape(-1)
        if self.unreal_layout and self.arch == "bighouse":  # bignet.py:77-96: one deconv per branch
            u["w1"][:, :, :, :A] = t(pick("pc_value", 0, "weight")).permute(0, 2, 3, 1)
            u["w1"][:, :, :, A:A + 1] = t(pick("pc_action", 0, "weight")).permute(0, 2, 3, 1)
            u["b1"][:A] = t(pick("pc_value", 0, "bias"))
            u["b1"][A] = t(pick("pc_action", 0, "bias")).view(())
        elif self.unreal_layout:
            u["w1"][:, :, :, :32] = t(pick("pc_value", 0, "weight")).permute(0, 2, 3, 1)
            u["w1"][:, :, :, 32:] = t(pick("pc_action", 0, "weight")).permute(0, 2, 3, 1)
            u["b1"][:32] = t(pick("pc_value", 0, "bias"))
            u["b1"][32:] = t(pick("pc_action", 0, "bias"))
            u["w2"][:32, :, :, :A] = t(pick("pc_value", 1, "weight")).permute(0, 2, 3, 1)
            u["w2"][32:, :, :, A:A + 1] = t(pick("pc_action", 1, "weight")).permute(0, 2, 3, 1)
            u["b2"][:A] = t(pick("pc_value", 1, "bias"))
            u["b2"][A] = t(pick("pc_action", 1, "bias")).view(())
        if self.unreal_layout:
            rw = t(pick("rp", 0, "weight"))
            if self.arch == "bighouse" and rw.shape[1] == 9 * 9 * 32 * 3 != u["rp_w"].shape[1]:
                # the reference module's rp as built (bignet.py:94), never usable at 84x84: keep
                # this policy's own rp (DESIGN row A23u), load everything else
                warnings.warn("BigHouseModel rp.weight takes %d inputs (bignet.py:94, 100x100 frames); this "
                              "%dx%d policy's rp takes %d: rp left at its initialisation, the rest loaded"
                              % (rw.shape[1], self.frame_hw[0], self.frame_hw[1], u["rp_w"].shape[1]))
            elif rw.shape[1] != u["rp_w"].shape[1]:
                raise ValueError("rp weight takes %d inputs, this frame size gives %d" % (rw.shape[1], u["rp_w"].shape[1]))
            else:
                u["rp_w"][:] = rw.view(3, 3, 32, o3[0], o3[1]).permute(0, 1, 3, 4, 2).reshape(3, -1)
                u["rp_b"][:3] = t(pick("rp", 0, "bias"))
        return flat.to(self.device)

    def to_reference(self, flat):
        """Flat params (or grads) -> dict in the reference's tensor shapes."""
        v = self.views(flat.detach().float().cpu())
        o3 = self.o3
        A = self.num_actions
        out = {}
        if self.arch == "bighouse":
            for i, (name, kk, ci, co) in enumerate((("conv1", 8, 3, 32), ("conv2", 4, 32, 64), ("conv3", 3, 64, 32))):
                w, b = v[name]
                out["conv_base.0.%d.weight" % (2 * i)] = w.reshape(co, kk, kk, ci).permute(0, 3, 1, 2).contiguous()
                out["conv_base.0.%d.bias" % (2 * i)] = b.clone()
        else:
            w, b = v["conv1"]
            out["shared_base.0.0.weight"] = w[:, :147].reshape(32, 7, 7, 3).permute(0, 3, 1, 2).contiguous()
            out["shared_base.0.0.bias"] = b.clone()
            w, b = v["conv2"]
            out["shared_base.0.2.weight"] = w.reshape(32, 4, 4, 32).permute(0, 3, 1, 2).contiguous()
            out["shared_base.0.2.bias"] = b.clone()
            w, b = v["conv3"]
            out["conv_base.0.0.weight"] = w.reshape(64, 4, 4, 64).permute(0, 3, 1, 2).contiguous()
            out["conv_base.0.0.bias"] = b.clone()
            w, b = v["conv4"]
            out["conv_base.0.2.weight"] = w.reshape(32, 64, 1, 1).clone()
            out["conv_base.0.2.bias"] = b.clone()
        w, b = v["fc"]
        out["conv_merge.0.1.weight"] = w.reshape(512, o3[0], o3[1], 32).permute(0, 3, 1, 2).reshape(512, -1).contiguous()
        out["conv_merge.0.1.bias"] = b.clone()
        w, b = v["head"]
        out["policy_logits.0.weight"] = w[:A].clone()
        out["policy_logits.0.bias"] = b[:A].clone()
        out["critic.0.weight"] = w[A:A + 1].clone()
        out["critic.0.bias"] = b[A:A + 1].clone()
        if self.lstm:
            L = self.lstm
            wcat, bih, bhh = v["lstm"]
            out["rnn.inner.weight_ih_l0"] = wcat[:, :L["lin"]].clone()
            out["rnn.inner.weight_hh_l0"] = wcat[:, L["xoff"]:].clone()
            out["rnn.inner.bias_ih_l0"] = bih.clone()
            out["rnn.inner.bias_hh_l0"] = bhh.clone()
        if self.aux_layout:
            w1, b1, w2, b2 = v["aux"]
            for hd, (name, c, o) in enumerate(AUX_HEADS):
                out["%s.0.1.weight" % name] = w1[:, :, :, 16 * hd:16 * hd + 16].permute(0, 3, 1, 2).contiguous()
                out["%s.0.1.bias" % name] = b1[16 * hd:16 * hd + 16].clone()
                out["%s.0.3.weight" % name] = w2[16 * hd:16 * hd + 16, :, :, o:o + c].permute(0, 3, 1, 2).contiguous()
                out["%s.0.3.bias" % name] = b2[o:o + c].clone()
        if self.unreal_layout:
            u, m = v["unreal"], PC_MAP
            out["pc_base.0.0.weight"] = u["pc_w"].view(m, m, 32, 512).permute(2, 0, 1, 3).reshape(PC_BASE, 512).clone()
            out["pc_base.0.0.bias"] = u["pc_b"].view(m, m, 32).permute(2, 0, 1).reshape(-1).clone()
        if self.unreal_layout and self.arch == "bighouse":
            out["pc_action.0.0.weight"] = u["w1"][:, :, :, A:A + 1].permute(0, 3, 1, 2).contiguous()
            out["pc_action.0.0.bias"] = u["b1"][A:A + 1].clone()
            out["pc_value.0.0.weight"] = u["w1"][:, :, :, :A].permute(0, 3, 1, 2).contiguous()
            out["pc_value.0.0.bias"] = u["b1"][:A].clone()
            out["rp.weight"] = u["rp_w"].view(3, 3, o3[0], o3[1], 32).permute(0, 1, 4, 2, 3).reshape(3, -1).clone()
            out["rp.bias"] = u["rp_b"][:3].clone()
        elif self.unreal_layout:
            out["pc_value.0.0.weight"] = u["w1"][:, :, :, :32].permute(0, 3, 1, 2).contiguous()
            out["pc_value.0.0.bias"] = u["b1"][:32].clone()
            out["pc_action.0.0.weight"] = u["w1"][:, :, :, 32:].permute(0, 3, 1, 2).contiguous()
            out["pc_action.0.0.bias"] = u["b1"][32:].clone()
            out["pc_value.0.2.weight"] = u["w2"][:32, :, :, :A].permute(0, 3, 1, 2).contiguous()
            out["pc_value.0.2.bias"] = u["b2"][:A].clone()
            out["pc_action.0.2.weight"] = u["w2"][32:, :, :, A:A + 1].permute(0, 3, 1, 2).contiguous()
            out["pc_action.0.2.bias"] = u["b2"][A:A + 1].clone()
            out["rp.1.weight"] = u["rp_w"].view(3, 3, o3[0], o3[1], 32).permute(0, 1, 4, 2, 3).reshape(3, -1).clone()
            out["rp.1.bias"] = u["rp_b"][:3].clone()
        return out

    # -- launches -------------------------------------------------------------------
    def workspace_floats(self, n):
        f = ctypes.c_int64()
        _lib.check(self.lib.vn_policy_workspace_floats(self._h, int(n), ctypes.byref(f)), "vn_policy_workspace_floats")
        return f.value

    def new_acts(self, capacity):
        return torch.empty(int(capacity) * self.act_floats, dtype=torch.float32, device=self.device)

    def x5(self, acts, capacity):
        """[capacity, 512] view of the conv_merge features in an activation store."""
        c = int(capacity)
        return acts[c * (self.act_floats - 512):c * self.act_floats].view(c, 512)

    def forward(self, params, frames, n, acts, capacity, offset, out, goals=None):
        """out=None (recurrent nets only): trunk only, features kept in acts. goals: a
        _lib.GoalRuns of this call's samples (goal-frame deduplication, vn_goal_runs)."""
        if goals is None:
            _lib.check(self.lib.vn_policy_forward(self._h, _lib.ptr(params), ctypes.byref(frames), int(n),
                                                  _lib.ptr(acts), int(capacity), int(offset), _lib.ptr(out),
                                                  _lib.stream_ptr(self.device)), "vn_policy_forward")
            return
        _lib.check(self.lib.vn_policy_forward_goals(self._h, _lib.ptr(params), ctypes.byref(frames), int(n),
                                                    _lib.ptr(acts), int(capacity), int(offset), _lib.ptr(out),
                                                    ctypes.byref(goals), _lib.stream_ptr(self.device)),
                   "vn_policy_forward_goals")

    def goal_runs_supported(self, n):
        """Whether forward / backward take goal runs for calls of n samples (84x84 / 174x174)."""
        ok = ctypes.c_int()
        _lib.check(self.lib.vn_policy_goal_runs_supported(self._h, int(n), ctypes.byref(ok)),
                   "vn_policy_goal_runs_supported")
        return bool(ok.value)

    def backward(self, params, frames, n, acts, capacity, dout, grads, workspace):
        _lib.check(self.lib.vn_policy_backward(self._h, _lib.ptr(params), ctypes.byref(frames), int(n), _lib.ptr(acts),
                                               int(capacity), _lib.ptr(dout), _lib.ptr(grads), _lib.ptr(workspace),
                                               _lib.stream_ptr(self.device)), "vn_policy_backward")

    def backward_ex(self, params, frames, n, acts, capacity, dout, dz5, dx4, grads, workspace, goals=None):
        P = _lib.ptr
        if goals is None:
            _lib.check(self.lib.vn_policy_backward_ex(self._h, P(params), ctypes.byref(frames), int(n), P(acts),
                                                      int(capacity), P(dout), P(dz5), P(dx4), P(grads), P(workspace),
                                                      _lib.stream_ptr(self.device)), "vn_policy_backward_ex")
            return
        _lib.check(self.lib.vn_policy_backward_goals(self._h, P(params), ctypes.byref(frames), int(n), P(acts),
                                                     int(capacity), P(dout), P(dz5), P(dx4), P(grads), P(workspace),
                                                     ctypes.byref(goals), _lib.stream_ptr(self.device)),
                   "vn_policy_backward_goals")

    # -- aux deconv heads ------------------------------------------------------------
    def aux_workspace_floats(self):
        f = ctypes.c_int64()
        _lib.check(self.lib.vn_aux_workspace_floats(self._h, ctypes.byref(f)), "vn_aux_workspace_floats")
        return f.value

    def aux_buffers(self, n):
        ah, aw = self.aux_layout["a_hw"]
        ph, pw = self.aux_layout["p_hw"]
        kw = dict(dtype=torch.float32, device=self.device)
        return torch.empty((n, ah, aw, 48), **kw), torch.empty((n, ph, pw, 8), **kw)

    def aux_forward(self, params, acts, capacity, n, a1, pred, workspace):
        P = _lib.ptr
        _lib.check(self.lib.vn_aux_forward(self._h, P(params), P(acts), int(capacity), int(n), P(a1), P(pred),
                                           P(workspace), _lib.stream_ptr(self.device)), "vn_aux_forward")

    def aux_target_table(self, depth, segmentation):
        """[rows, PH, PW, 4] float targets from the env's aux arena (depth, segmentation)."""
        rows, H, W = depth.shape[:3]
        ph, pw = self.aux_layout["p_hw"]
        table = torch.empty((rows, ph, pw, 4), dtype=torch.float32, device=self.device)
        _lib.check(self.lib.vn_aux_target_table(self._h, _lib.ptr(depth), _lib.ptr(segmentation), int(H), int(W),
                                                int(rows), _lib.ptr(table), _lib.stream_ptr(self.device)),
                   "vn_aux_target_table")
        return table

    def aux_loss_grad(self, pred, n, targets, weight, dpred, stats):
        P = _lib.ptr
        _lib.check(self.lib.vn_aux_loss_grad(self._h, P(pred), int(n), ctypes.byref(targets), ctypes.c_float(weight),
                                             P(dpred), P(stats), _lib.stream_ptr(self.device)), "vn_aux_loss_grad")

    def aux_forward_loss_grad(self, params, acts, capacity, n, a1, pred, targets, weight, dpred, stats, workspace):
        """aux_forward + aux_loss_grad with the loss fused into the second head layer (pred is
        scratch: written only for maps too large for the fused kernel)."""
        P = _lib.ptr
        _lib.check(self.lib.vn_aux_forward_loss_grad(self._h, P(params), P(acts), int(capacity), int(n), P(a1),
                                                     P(pred), ctypes.byref(targets), ctypes.c_float(weight), P(dpred),
                                                     P(stats), P(workspace), _lib.stream_ptr(self.device)),
                   "vn_aux_forward_loss_grad")

    def aux_backward(self, params, acts, capacity, n, a1, dpred, grads, dx4, workspace):
        P = _lib.ptr
        _lib.check(self.lib.vn_aux_backward(self._h, P(params), P(acts), int(capacity), int(n), P(a1), P(dpred),
                                            P(grads), P(dx4), P(workspace), _lib.stream_ptr(self.device)),
                   "vn_aux_backward")

    # -- UNREAL heads (goal.py:94-133) ------------------------------------------------
    def pc_workspace_floats(self):
        f = ctypes.c_int64()
        _lib.check(self.lib.vn_pc_workspace_floats(self._h, ctypes.byref(f)), "vn_pc_workspace_floats")
        return f.value

    def pc_buffers(self, n, with_q=True):
        """pcb [n,9,9,32], a1 [n,20,20,64], p2 [n,42,42,8], q [n,42,42,A] (None without q);
        BigHouseModel: a1 None, p2 [n,20,20,8], q [n,20,20,A]."""
        kw = dict(dtype=torch.float32, device=self.device)
        s = self.pc_side
        a1 = None if self.arch == "bighouse" else torch.empty((n, PC_A1, PC_A1, 64), **kw)
        return (torch.empty((n, PC_MAP, PC_MAP, 32), **kw), a1, torch.empty((n, s, s, 8), **kw),
                torch.empty((n, s, s, self.num_actions), **kw) if with_q else None)

    def pc_forward(self, params, h, n, pcb, a1, p2, q, workspace):
        P = _lib.ptr
        _lib.check(self.lib.vn_pc_forward(self._h, P(params), P(h), int(n), P(pcb), P(a1), P(p2), P(q), P(workspace),
                                          _lib.stream_ptr(self.device)), "vn_pc_forward")

    def pc_backward(self, params, h, n, pcb, a1, p2, dq, grads, dh, workspace, accumulate=False):
        P = _lib.ptr
        _lib.check(self.lib.vn_pc_backward(self._h, P(params), P(h), int(n), P(pcb), P(a1), P(p2), P(dq), P(grads),
                                           P(dh), int(bool(accumulate)), P(workspace), _lib.stream_ptr(self.device)),
                   "vn_pc_backward")

    def rp_forward(self, params, x, n, out):
        P = _lib.ptr
        _lib.check(self.lib.vn_rp_forward(self._h, P(params), P(x), int(n), P(out), _lib.stream_ptr(self.device)),
                   "vn_rp_forward")

    def rp_backward(self, params, x, n, dout, grads, dx, workspace):
        P = _lib.ptr
        _lib.check(self.lib.vn_rp_backward(self._h, P(params), P(x), int(n), P(dout), P(grads), P(dx), P(workspace),
                                           _lib.stream_ptr(self.device)), "vn_rp_backward")

    def x4(self, acts, capacity):
        """[capacity, h3*w3*32] view of conv_base's output (X4) in an activation store."""
        c = int(capacity)
        s4 = self.fc_in
        off = c * (self.act_floats - 512 - s4)
        return acts[off:off + c * s4].view(c, s4)

    def backward_trunk(self, params, frames, n, acts, capacity, dz5, grads, workspace):
        _lib.check(self.lib.vn_policy_backward_trunk(self._h, _lib.ptr(params), ctypes.byref(frames), int(n),
                                                     _lib.ptr(acts), int(capacity), _lib.ptr(dz5), _lib.ptr(grads),
                                                     _lib.ptr(workspace), _lib.stream_ptr(self.device)),
                   "vn_policy_backward_trunk")

    # -- recurrent core -------------------------------------------------------------
    def lstm_workspace_floats(self, T, E):
        f = ctypes.c_int64()
        _lib.check(self.lib.vn_lstm_workspace_floats(self._h, int(T), int(E), ctypes.byref(f)),
                   "vn_lstm_workspace_floats")
        return f.value

    def lstm_step(self, params, E, x5, lra, mask, h_prev, c_prev, xcat, gates, acts, c_out, h_out):
        P = _lib.ptr
        _lib.check(self.lib.vn_lstm_forward_step(self._h, P(params), int(E), P(x5), P(lra), P(mask), P(h_prev),
                                                 P(c_prev), P(xcat), P(gates), P(acts), P(c_out), P(h_out),
                                                 _lib.stream_ptr(self.device)), "vn_lstm_forward_step")

    def heads(self, params, feat, n, out):
        _lib.check(self.lib.vn_policy_heads(self._h, _lib.ptr(params), _lib.ptr(feat), int(n), _lib.ptr(out),
                                            _lib.stream_ptr(self.device)), "vn_policy_heads")

    def lstm_backward(self, params, T, E, dout, h_all, xcat_all, acts_all, c_all, c_init, mask_all, x5_all, dz5_all,
                      grads, workspace, dh_extra=None, extra_envs=0):
        """dh_extra [T, extra_envs, 512]: another head's gradient w.r.t. h of the first
        extra_envs envs (pixel control), added to the policy heads' (vn_lstm_backward_ex)."""
        P = _lib.ptr
        if dh_extra is None:
            _lib.check(self.lib.vn_lstm_backward(self._h, P(params), int(T), int(E), P(dout), P(h_all), P(xcat_all),
                                                 P(acts_all), P(c_all), P(c_init), P(mask_all), P(x5_all), P(dz5_all),
                                                 P(grads), P(workspace), _lib.stream_ptr(self.device)),
                       "vn_lstm_backward")
            return
        _lib.check(self.lib.vn_lstm_backward_ex(self._h, P(params), int(T), int(E), P(dout), P(h_all), P(xcat_all),
                                                P(acts_all), P(c_all), P(c_init), P(mask_all), P(x5_all), P(dh_extra),
                                                int(extra_envs), P(dz5_all), P(grads), P(workspace),
                                                _lib.stream_ptr(self.device)), "vn_lstm_backward_ex")


def _lstm_param(sd, suffix):
    keys = [k for k in sd if k.endswith(suffix)]
    if len(keys) != 1:
        raise KeyError("expected one LSTM parameter *%s in the state dict, found %s" % (suffix, keys))
    return sd[keys[0]]


class _ReferenceNames:
    """Resolve reference parameter names with or without the TimeDistributed/Sequential
    nesting (e.g. 'shared_base.0.0.weight' or 'shared_base.module.0.weight')."""

    def __init__(self, sd):
        self.sd = {k: v for k, v in sd.items()}

    def __call__(self, module, index, kind):
        cands = []
        for k in self.sd:
            parts = k.split(".")
            if parts[0] != module or parts[-1] != kind:
                continue
            nums = [int(p) for p in parts[1:-1] if re.fullmatch(r"\d+", p)]
            cands.append((nums, k))
        cands.sort()
        if index >= len(cands):
            raise KeyError("no %s[%d].%s in the state dict" % (module, index, kind))
        return self.sd[cands[index][1]]


class _GoalNavFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, params, image, goal, net):
        net.check_frames(image, goal)
        n = image.shape[0]
        acts = net.new_acts(n)
        out = torch.empty((n, OUT_LD), dtype=torch.float32, device=params.device)
        frames = frames_from_batch(image, goal)
        net.forward(params, frames, n, acts, n, 0, out)
        ctx.save_for_backward(params, image, goal, acts)
        ctx.net = net
        return out[:, : net.num_actions + 1]

    @staticmethod
    def backward(ctx, dout):
        params, image, goal, acts = ctx.saved_tensors
        net = ctx.net
        n = image.shape[0]
        d = torch.zeros((n, OUT_LD), dtype=torch.float32, device=params.device)
        d[:, : net.num_actions + 1] = dout
        # zeros: the backward writes the trunk and head blocks only; an aux / UNREAL policy's
        # other blocks take no gradient from this output (uninitialised memory there was
        # returned as their gradient until round 6: tools/nan_stress.py found ~1/256 of them
        # non-finite)
        grads = torch.zeros_like(params)
        ws = torch.empty(net.workspace_floats(n), dtype=torch.float32, device=params.device)
        net.backward(params, frames_from_batch(image, goal), n, acts, n, d, grads, ws)
        return grads, None, None, None


class _RecurrentGoalNavFunction(torch.autograd.Function):
    """Trunk over all T*B samples (time-major rows t*B + b), LSTM steps, heads on h.
    Gradients reach the parameters only: BPTT stops at the states entering the sequence
    (and lra / masks are inputs), as in a truncated-BPTT rollout."""

    @staticmethod
    def forward(ctx, params, image, goal, lra, masks, h0, c0, net, T, B):
        net.check_frames(image, goal)
        n = T * B
        if image.shape[0] != n or lra.shape != (n, net.num_actions + 1) or masks.shape != (T, B) or \
                h0.shape != (B, 512) or c0.shape != (B, 512):
            raise ValueError("recurrent inputs do not match T=%d, B=%d" % (T, B))
        dev = params.device
        acts = net.new_acts(n)
        frames = frames_from_batch(image, goal)
        net.forward(params, frames, n, acts, n, 0, None)
        x5 = net.x5(acts, n)
        L = net.lstm
        xcat = torch.empty((n, L["xcat"]), dtype=torch.float32, device=dev)
        gates = torch.empty((B, 2048), dtype=torch.float32, device=dev)
        la = torch.empty((n, 2048), dtype=torch.float32, device=dev)
        c_all = torch.empty((n, 512), dtype=torch.float32, device=dev)
        h_all = torch.empty((n, 512), dtype=torch.float32, device=dev)
        hp, cp = h0, c0
        for t in range(T):
            sl = slice(t * B, (t + 1) * B)
            net.lstm_step(params, B, x5[sl], lra[sl], masks[t], hp, cp, xcat[sl], gates, la[sl], c_all[sl], h_all[sl])
            hp, cp = h_all[sl], c_all[sl]
        out = torch.empty((n, OUT_LD), dtype=torch.float32, device=dev)
        net.heads(params, h_all, n, out)
        ctx.save_for_backward(params, image, goal, acts, xcat, la, c_all, h_all, c0, masks)
        ctx.net, ctx.T, ctx.B = net, T, B
        hT, cT = h_all[(T - 1) * B:].clone(), c_all[(T - 1) * B:].clone()
        ctx.mark_non_differentiable(hT, cT)
        return out[:, : net.num_actions + 1], hT, cT

    @staticmethod
    def backward(ctx, dout, _dh, _dc):
        params, image, goal, acts, xcat, la, c_all, h_all, c0, masks = ctx.saved_tensors
        net, T, B = ctx.net, ctx.T, ctx.B
        n = T * B
        dev = params.device
        d = torch.zeros((n, OUT_LD), dtype=torch.float32, device=dev)
        d[:, : net.num_actions + 1] = dout
        grads = torch.zeros_like(params)
        dz5 = torch.empty((n, 512), dtype=torch.float32, device=dev)
        ws = torch.empty(net.lstm_workspace_floats(T, B), dtype=torch.float32, device=dev)
        net.lstm_backward(params, T, B, d, h_all, xcat, la, c_all, c0, masks, net.x5(acts, n), dz5, grads, ws)
        del ws
        ws = torch.empty(net.workspace_floats(n), dtype=torch.float32, device=dev)
        net.backward_trunk(params, frames_from_batch(image, goal), n, acts, n, dz5, grads, ws)
        return (grads,) + (None,) * 9


class _AuxDeconvFunction(torch.autograd.Function):
    """Trunk to conv_base (X4) + the three deconv heads; gradients reach the parameters."""

    @staticmethod
    def forward(ctx, params, image, goal, net):
        net.check_frames(image, goal)
        n = image.shape[0]
        dev = params.device
        acts = net.new_acts(n)
        frames = frames_from_batch(image, goal)
        out = None if net.recurrent else torch.empty((n, OUT_LD), dtype=torch.float32, device=dev)
        net.forward(params, frames, n, acts, n, 0, out)
        a1, pred = net.aux_buffers(n)
        ws = torch.empty(net.aux_workspace_floats(), dtype=torch.float32, device=dev)
        net.aux_forward(params, acts, n, n, a1, pred, ws)
        ctx.save_for_backward(params, image, goal, acts, a1)
        ctx.net = net
        return pred

    @staticmethod
    def backward(ctx, dpred):
        params, image, goal, acts, a1 = ctx.saved_tensors
        net = ctx.net
        n = image.shape[0]
        dev = params.device
        grads = torch.zeros_like(params)
        dx4 = torch.empty((n, net.fc_in), dtype=torch.float32, device=dev)
        ws = torch.empty(net.aux_workspace_floats(), dtype=torch.float32, device=dev)
        net.aux_backward(params, acts, n, n, a1.clone(), dpred.contiguous(), grads, dx4, ws)
        dz5 = torch.zeros((n, 512), dtype=torch.float32, device=dev)  # heads / LSTM take no gradient here
        ws = torch.empty(net.workspace_floats(n), dtype=torch.float32, device=dev)
        net.backward_ex(params, frames_from_batch(image, goal), n, acts, n, None, dz5, dx4, grads, ws)
        return grads, None, None, None


class _RecurrentFeaturesFunction(torch.autograd.Function):
    """_forward_base (goal.py:83-92) with the recurrent core: the LSTM outputs h [T*B, 512]
    (time-major rows) of the trunk + LSTM; the backward takes dL/dh into the LSTM backward
    (vn_lstm_backward_ex, no policy-head gradient) and the trunk backward."""

    @staticmethod
    def forward(ctx, params, image, goal, lra, masks, h0, c0, net, T, B):
        net.check_frames(image, goal)
        n = T * B
        dev = params.device
        acts = net.new_acts(n)
        frames = frames_from_batch(image, goal)
        net.forward(params, frames, n, acts, n, 0, None)
        x5 = net.x5(acts, n)
        L = net.lstm
        xcat = torch.empty((n, L["xcat"]), dtype=torch.float32, device=dev)
        gates = torch.empty((B, 2048), dtype=torch.float32, device=dev)
        la = torch.empty((n, 2048), dtype=torch.float32, device=dev)
        c_all = torch.empty((n, 512), dtype=torch.float32, device=dev)
        h_all = torch.empty((n, 512), dtype=torch.float32, device=dev)
        hp, cp = h0, c0
        for t in range(T):
            sl = slice(t * B, (t + 1) * B)
            net.lstm_step(params, B, x5[sl], lra[sl], masks[t], hp, cp, xcat[sl], gates, la[sl], c_all[sl], h_all[sl])
            hp, cp = h_all[sl], c_all[sl]
        ctx.save_for_backward(params, image, goal, acts, xcat, la, c_all, h_all, c0, masks)
        ctx.net, ctx.T, ctx.B = net, T, B
        hT, cT = h_all[(T - 1) * B:].clone(), c_all[(T - 1) * B:].clone()
        ctx.mark_non_differentiable(hT, cT)
        return h_all.clone(), hT, cT

    @staticmethod
    def backward(ctx, dh, _dh, _dc):
        params, image, goal, acts, xcat, la, c_all, h_all, c0, masks = ctx.saved_tensors
        net, T, B = ctx.net, ctx.T, ctx.B
        n = T * B
        dev = params.device
        grads = torch.zeros_like(params)
        dz5 = torch.empty((n, 512), dtype=torch.float32, device=dev)
        zero_out = torch.zeros((n, OUT_LD), dtype=torch.float32, device=dev)
        ws = torch.empty(net.lstm_workspace_floats(T, B), dtype=torch.float32, device=dev)
        net.lstm_backward(params, T, B, zero_out, h_all, xcat, la, c_all, c0, masks, net.x5(acts, n), dz5, grads, ws,
                          dh_extra=dh.contiguous(), extra_envs=B)
        del ws
        ws = torch.empty(net.workspace_floats(n), dtype=torch.float32, device=dev)
        net.backward_trunk(params, frames_from_batch(image, goal), n, acts, n, dz5, grads, ws)
        return (grads,) + (None,) * 9


class _PixelControlFunction(torch.autograd.Function):
    """pc_base + pc_value / pc_action + combination (goal.py:133-136) on feature rows h."""

    @staticmethod
    def forward(ctx, params, h, net):
        n = h.shape[0]
        h = h.contiguous()
        pcb, a1, p2, q = net.pc_buffers(n)
        ws = torch.empty(net.pc_workspace_floats(), dtype=torch.float32, device=params.device)
        net.pc_forward(params, h, n, pcb, a1, p2, q, ws)
        ctx.save_for_backward(params, h, pcb, a1, p2)
        ctx.net = net
        return q

    @staticmethod
    def backward(ctx, dq):
        params, h, pcb, a1, p2 = ctx.saved_tensors
        net = ctx.net
        n = h.shape[0]
        grads = torch.zeros_like(params)
        dh = torch.empty_like(h)
        ws = torch.empty(net.pc_workspace_floats(), dtype=torch.float32, device=params.device)
        net.pc_backward(params, h, n, pcb.clone(), None if a1 is None else a1.clone(), p2.clone(), dq.contiguous(), grads,
                        dh, ws)
        return grads, dh, None


class _RewardPredictionFunction(torch.autograd.Function):
    """reward_prediction (goal.py:121-129): the trunk to conv_base on the 3 frames of each
    sample (rows b*3 + k), rp on their concatenated maps; gradients reach the parameters."""

    @staticmethod
    def forward(ctx, params, image, goal, net):
        net.check_frames(image, goal)
        n = image.shape[0]
        R = n // 3
        dev = params.device
        acts = net.new_acts(n)
        frames = frames_from_batch(image, goal)
        out = None if net.recurrent else torch.empty((n, OUT_LD), dtype=torch.float32, device=dev)
        net.forward(params, frames, n, acts, n, 0, out)
        x = net.x4(acts, n).reshape(R, 3 * net.fc_in)
        logits = torch.empty((R, 4), dtype=torch.float32, device=dev)
        net.rp_forward(params, x, R, logits)
        ctx.save_for_backward(params, image, goal, acts)
        ctx.net = net
        return logits[:, :3]

    @staticmethod
    def backward(ctx, dlogits):
        params, image, goal, acts = ctx.saved_tensors
        net = ctx.net
        n = image.shape[0]
        R = n // 3
        dev = params.device
        grads = torch.zeros_like(params)
        dout = torch.zeros((R, 4), dtype=torch.float32, device=dev)
        dout[:, :3] = dlogits
        dx = torch.empty((R, 3 * net.fc_in), dtype=torch.float32, device=dev)
        ws = torch.empty(net.pc_workspace_floats(), dtype=torch.float32, device=dev)
        net.rp_backward(params, net.x4(acts, n).reshape(R, -1), R, dout, grads, dx, ws)
        dz5 = torch.zeros((n, 512), dtype=torch.float32, device=dev)  # heads / LSTM take no gradient here
        ws = torch.empty(net.workspace_floats(n), dtype=torch.float32, device=dev)
        net.backward_ex(params, frames_from_batch(image, goal), n, acts, n, None, dz5, dx.view(n, net.fc_in), grads, ws)
        return grads, None, None, None


class GoalNavPolicy(torch.nn.Module):
    """Drop-in for BigGoalHouseModel's trunk + heads (see module docstring)."""

    _ARCH = "goal"

    def __init__(self, num_inputs=3, num_outputs=4, frame_hw=(84, 84), device=None, seed=0, recurrent=False,
                 aux=False, unreal=False):
        super().__init__()
        if num_inputs != 3:
            raise ValueError("frames are RGB (num_inputs=3)")
        self.net = PolicyNet(frame_hw, num_outputs, device, recurrent=recurrent, aux=aux, arch=self._ARCH,
                             unreal=unreal)
        self.pc_cell_size = 4  # goal.py:72
        self.deconv_cell_size = 4  # goal.py:70,148
        self.params = torch.nn.Parameter(self.net.init_params(seed))
        self.lstm_layers, self.lstm_hidden_size = 1, 512  # goal.py:61-62 (state shape contract)

    @classmethod
    def wrap(cls, net, params):
        """A policy over an existing PolicyNet whose parameter aliases ``params`` (the flat
        device buffer of a trainer: no copy, the kernels' updates are seen here)."""
        if net.arch != cls._ARCH:
            cls = BigHousePolicy if net.arch == "bighouse" else GoalNavPolicy
        self = cls.__new__(cls)
        torch.nn.Module.__init__(self)
        self.net = net
        self.deconv_cell_size = 4
        self.params = torch.nn.Parameter(params)
        self.lstm_layers, self.lstm_hidden_size = 1, 512
        return self

    def initial_states(self, batch_size):
        return tuple(torch.zeros([batch_size, self.lstm_layers, self.lstm_hidden_size], dtype=torch.float32)
                     for _ in range(2))

    def load_reference_state_dict(self, sd):
        with torch.no_grad():
            self.params.copy_(self.net.from_reference(sd, init=self.params))
        return self

    def reference_state_dict(self):
        return self.net.to_reference(self.params)

    def forward(self, inputs, masks=None, states=None):
        observations, _last_reward_action = inputs if isinstance(inputs, tuple) and len(inputs) == 2 and \
            isinstance(inputs[0], (tuple, list)) else (inputs, None)
        image, goal = observations[0], observations[1]
        if self.net.recurrent:
            return self._forward_recurrent(image, goal, _last_reward_action, masks, states)
        lead = image.shape[:2]
        dev = self.params.device
        if image.dtype == torch.uint8:   # env frames [B,T,H,W,3]
            img = image.to(dev).reshape(-1, *image.shape[2:]).contiguous()
            gl = goal.to(dev).reshape(-1, *goal.shape[2:]).contiguous()
        else:                            # reference wrapper output [B,T,3,H,W] float
            img = image.to(dev).reshape(-1, *image.shape[2:]).float().contiguous()
            gl = goal.to(dev).reshape(-1, *goal.shape[2:]).float().contiguous()
        out = _GoalNavFunction.apply(self.params, img, gl, self.net)
        A = self.net.num_actions
        return [out[:, :A].reshape(*lead, A), out[:, A:A + 1].reshape(*lead, 1), states]

    def _forward_recurrent(self, image, goal, lra, masks, states):
        """goal.py:84-92 with the recurrent core: inputs [B,T,...] batch-first."""
        B, T = image.shape[:2]
        dev = self.params.device
        A = self.net.num_actions

        def time_major(x, dtype=None):
            x = x.to(dev).transpose(0, 1)
            return x.reshape(T * B, *x.shape[2:]).to(dtype or x.dtype).contiguous()

        if image.dtype == torch.uint8:
            img, gl = time_major(image), time_major(goal)
        else:
            img, gl = time_major(image, torch.float32), time_major(goal, torch.float32)
        if lra is None:
            lra = torch.zeros((B, T, A + 1), dtype=torch.float32, device=dev)
        if lra.shape[-1] != A + 1:
            raise ValueError("last_reward_action must be [B,T,%d]" % (A + 1))
        lr = time_major(lra, torch.float32)
        m = torch.ones((B, T), dtype=torch.float32, device=dev) if masks is None else masks
        m = m.to(dev).reshape(B, T).to(torch.float32).t().contiguous()
        if states is None:
            states = self.initial_states(B)
        h0 = states[0].to(dev, torch.float32).reshape(B, 512).contiguous()
        c0 = states[1].to(dev, torch.float32).reshape(B, 512).contiguous()
        out, hT, cT = _RecurrentGoalNavFunction.apply(self.params, img, gl, lr, m, h0, c0, self.net, T, B)
        out = out.view(T, B, A + 1).transpose(0, 1)
        return [out[..., :A], out[..., A:A + 1], (hT.view(B, 1, 512), cT.view(B, 1, 512))]

    def value_prediction(self, inputs, masks=None, states=None):
        """BigGoalHouseModel.value_prediction (goal.py:135-138): the critic over the recurrent
        features of ``inputs`` -> (value [B,T,1], states). The same HIP forward as ``forward``
        (the critic is one column of the fused heads product), so the value is bit-identical
        to forward's and its gradient flows through the same backward."""
        _logits, value, states = self.forward(inputs, masks, states)
        return value, states

    def _time_major_inputs(self, inputs, masks, states):
        observations, lra = inputs
        image, goal = observations[0], observations[1]
        B, T = image.shape[:2]
        dev = self.params.device
        A = self.net.num_actions

        def time_major(x, dtype=None):
            x = x.to(dev).transpose(0, 1)
            return x.reshape(T * B, *x.shape[2:]).to(dtype or x.dtype).contiguous()

        fdt = None if image.dtype == torch.uint8 else torch.float32
        img, gl = time_major(image, fdt), time_major(goal, fdt)
        if lra is None:
            lra = torch.zeros((B, T, A + 1), dtype=torch.float32, device=dev)
        lr = time_major(lra, torch.float32)
        m = torch.ones((B, T), dtype=torch.float32, device=dev) if masks is None else masks
        m = m.to(dev).reshape(B, T).to(torch.float32).t().contiguous()
        if states is None:
            states = self.initial_states(B)
        h0 = states[0].to(dev, torch.float32).reshape(B, 512).contiguous()
        c0 = states[1].to(dev, torch.float32).reshape(B, 512).contiguous()
        return img, gl, lr, m, h0, c0, T, B

    def pixel_control(self, inputs, masks=None, states=None):
        """BigGoalHouseModel.pixel_control (goal.py:131-137): Q maps [B,T,A,42,42] =
        pc_value + pc_action - mean(pc_action) over the recurrent features, and the states."""
        if not (self.net.unreal and self.net.recurrent):
            raise ValueError("pixel_control needs GoalNavPolicy(recurrent=True, unreal=True)")
        img, gl, lr, m, h0, c0, T, B = self._time_major_inputs(inputs, masks, states)
        h, hT, cT = _RecurrentFeaturesFunction.apply(self.params, img, gl, lr, m, h0, c0, self.net, T, B)
        q = _PixelControlFunction.apply(self.params, h, self.net)  # [T*B, 42, 42, A] (20x20: BigHouseModel)
        q = q.view(T, B, *q.shape[1:]).permute(1, 0, 4, 2, 3)
        return q, (hT.view(B, 1, 512), cT.view(B, 1, 512))

    def reward_prediction(self, inputs):
        """BigGoalHouseModel.reward_prediction (goal.py:121-129): logits [B,3] from the
        conv_base maps of the B samples' 3 frames (observations [B,3,...])."""
        if not self.net.unreal:
            raise ValueError("reward_prediction needs GoalNavPolicy(unreal=True)")
        observations = inputs[0] if isinstance(inputs, tuple) and len(inputs) == 2 and \
            isinstance(inputs[0], (tuple, list)) else inputs
        image, goal = observations[0], observations[1]
        if image.shape[1] != 3:
            raise ValueError("reward_prediction takes 3 frames per sample ([B,3,...])")
        dev = self.params.device
        fdt = None if image.dtype == torch.uint8 else torch.float32
        img = image.to(dev).reshape(-1, *image.shape[2:]).to(fdt or image.dtype).contiguous()
        gl = goal.to(dev).reshape(-1, *goal.shape[2:]).to(fdt or goal.dtype).contiguous()
        return _RewardPredictionFunction.apply(self.params, img, gl, self.net)

    def forward_deconv(self, inputs, masks=None, states=None):
        """AuxiliaryBigGoalHouseModel.forward_deconv (goal.py:177-189): (depth [B,T,1,h,w],
        mask [B,T,3,h,w], goal mask [B,T,3,h,w]) from conv_base's map, states unchanged."""
        if not self.net.aux:
            raise ValueError("forward_deconv needs GoalNavPolicy(aux=True)")
        observations = inputs[0] if isinstance(inputs, tuple) and len(inputs) == 2 and \
            isinstance(inputs[0], (tuple, list)) else inputs
        image, goal = observations[0], observations[1]
        lead = image.shape[:2]
        dev = self.params.device
        if image.dtype == torch.uint8:
            img = image.to(dev).reshape(-1, *image.shape[2:]).contiguous()
            gl = goal.to(dev).reshape(-1, *goal.shape[2:]).contiguous()
        else:
            img = image.to(dev).reshape(-1, *image.shape[2:]).float().contiguous()
            gl = goal.to(dev).reshape(-1, *goal.shape[2:]).float().contiguous()
        pred = _AuxDeconvFunction.apply(self.params, img, gl, self.net)  # [n, h, w, 8] NHWC
        p = pred.permute(0, 3, 1, 2)
        h, w = p.shape[-2:]
        heads = tuple(p[:, o:o + c].reshape(*lead, c, h, w) for _, c, o in AUX_HEADS)
        return heads, states


class BigHousePolicy(GoalNavPolicy):
    """Drop-in for BigHouseModel (models/bignet.py:26-75): ``forward(inputs, masks, states)``
    with ``inputs = (observations, last_reward_action)`` and observations ONE image tensor
    ([B,T,84,84,3] uint8 or [B,T,3,84,84] float), Nature-CNN trunk (Conv k8s4 -> k4s2 -> k3,
    Linear(7*7*32, 512)) on the HIP kernels, then the heads (recurrent=True: the LSTM core)."""

    _ARCH = "bighouse"

    def __init__(self, num_inputs=3, num_outputs=4, device=None, seed=0, recurrent=True, unreal=False):
        super().__init__(num_inputs, num_outputs, (84, 84), device, seed, recurrent=recurrent, unreal=unreal)

    @staticmethod
    def _both_slots(inputs):
        observations, last_reward_action = inputs if isinstance(inputs, tuple) and len(inputs) == 2 \
            else (inputs, None)
        # the image feeds both frame slots; the BigHouse kernels read only the first
        return (observations, observations), last_reward_action

    def forward(self, inputs, masks=None, states=None):
        return super().forward(self._both_slots(inputs), masks, states)

    def pixel_control(self, inputs, masks=None, states=None):
        """BigHouseModel.pixel_control (bignet.py:105-111): Q maps [B,T,A,20,20] = pc_value +
        pc_action - mean(pc_action) (one ConvTranspose2d(32, ., 4, 2) + ReLU per branch on
        pc_base's 9x9 map) over the recurrent features, and the states."""
        return super().pixel_control(self._both_slots(inputs), masks, states)

    def reward_prediction(self, inputs):
        """BigHouseModel.reward_prediction (bignet.py:98-103): logits [B,3] of the conv_base
        maps of each sample's 3 frames (observations [B,3,...]); rp takes 3 * 7*7*32 inputs at
        84x84 (bignet.py:96 writes 9*9*32*3, which fits 100x100 frames only)."""
        return super().reward_prediction(self._both_slots(inputs))

    def forward_deconv(self, inputs, masks=None, states=None):
        raise NotImplementedError("BigHouseModel has no deconv heads (bignet.py)")

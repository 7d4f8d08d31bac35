"""Where the driver's short bench window loses time: host microseconds per
VectorEnv.step call (enqueue rate, the GPU kept busy), and the bench-style timed window at
K steps (barrier + synchronize on both sides) against the HIP-event device time, for
several K and both call paths (validated vs. cached buffers). Prints one JSON line.

    python tools/host_overhead.py [--envs 4096] [--scenes 20]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "a2cat-vn-pytorch_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--scenes", type=int, default=20)
    a = ap.parse_args()
    import vnav
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    scenes = [vnav.synthetic_scene(k) for k in range(a.scenes)]
    E = a.envs
    env = vnav.VectorEnv(scenes, E, seed=1000, device=dev)
    out = dict(image=torch.empty((E,) + env.frame_shape, dtype=torch.uint8, device=dev),
               goal=torch.empty((E,) + env.frame_shape, dtype=torch.uint8, device=dev),
               reward=torch.empty(E, dtype=torch.float32, device=dev),
               done=torch.empty(E, dtype=torch.bool, device=dev),
               state=torch.empty(E, dtype=torch.int32, device=dev))
    n = 2000
    acts = torch.empty((n, E), dtype=torch.int32, device=dev)
    for t in range(n):
        env.random_actions(t, out=acts[t])
    views = list(acts.unbind(0))
    for t in range(20):
        env.step(views[t], out=out)
    torch.cuda.synchronize()
    res = {}
    # host enqueue cost: time the loop without waiting (the queue absorbs the launches)
    for label, fn in (("step", lambda t: env.step(views[t], out=out)),
                      ("step_noout", lambda t: env.step(views[t], gather=False))):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(200):
            fn(t)
        res["host_us_per_call_" + label] = (time.perf_counter() - t0) / 200 * 1e6
        torch.cuda.synchronize()
    # bench-style windows
    for K, W in ((20, 5), (100, 5), (1000, 50)):
        for t in range(W):
            env.step(views[t], out=out)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ev0.record()
        ta = time.perf_counter()
        for k in range(K):
            env.step(views[W + k], out=out)
        tb = time.perf_counter()
        ev1.record()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        res["K%d" % K] = {"ms_per_step": el / K * 1e3, "kernel_ms": ev0.elapsed_time(ev1) / K,
                          "host_enqueue_ms": (tb - ta) * 1e3, "window_ms": el * 1e3,
                          "first_record_us": (ta - t0) * 1e6}
    # empty-window latency: synchronize -> event record -> synchronize
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    torch.cuda.synchronize(dev)
    res["empty_window_us"] = (time.perf_counter() - t0) * 1e6
    print(json.dumps(res))


if __name__ == "__main__":
    main()

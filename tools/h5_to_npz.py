"""Convert a reference h5 scene (graph/util.py:222-227 layout) to the .npz vnav.scenes.load_npz
reads, optionally resizing the frames offline.

    /opt/conda/bin/python3.9 tools/h5_to_npz.py SCENE.h5 OUT.npz [--size H W]

Needs h5py (and scikit-image for --size), which the Anaconda interpreter of this image has;
the product itself never imports them. Datasets copied: graph, shortest_path_distance,
observation, location (if present). resnet_feature is not read by the env and is dropped.

--size H W applies the reference's per-step preprocessing once, offline:
skimage.transform.resize(frame, (H, W), anti_aliasing=True) (cached.py:62-64), whose
float64 output in [0, 1] is stored as round(255 x) uint8 so the scene cache stays 1 B per
channel; the policy's u8/255 input conversion then differs from the reference's float frame
by at most 0.5/255 (tests/test_ingest.py pins this against the reference's own output).
Frames are converted one at a time (scenes larger than memory stream through).
"""
import argparse
import sys

import numpy as np


def convert(src, dst, size=None):
    import h5py
    with h5py.File(src, "r") as f:
        graph = f["graph"][()].astype(np.int64)
        spd = f["shortest_path_distance"][()].astype(np.int64)
        obs_ds = f["observation"]
        n = obs_ds.shape[0]
        out = {"graph": graph, "shortest_path_distance": spd}
        if "location" in f:
            out["location"] = f["location"][()]
        if size is None or tuple(obs_ds.shape[1:3]) == tuple(size):
            out["observation"] = obs_ds[()].astype(np.uint8)
        else:
            from skimage.transform import resize
            frames = np.empty((n,) + tuple(size) + obs_ds.shape[3:], dtype=np.uint8)
            for i in range(n):
                x = resize(obs_ds[i], tuple(size), anti_aliasing=True)
                frames[i] = np.clip(np.rint(x * 255.0), 0, 255).astype(np.uint8)
            out["observation"] = frames
    if graph.shape != (n, 4) or spd.shape != (n, n):
        raise ValueError("%s: graph must be [N,4] and shortest_path_distance [N,N]" % src)
    np.savez(dst, **out)
    return out


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    p.add_argument("src")
    p.add_argument("dst")
    p.add_argument("--size", type=int, nargs=2, metavar=("H", "W"))
    a = p.parse_args(argv)
    out = convert(a.src, a.dst, a.size)
    print("%s: %d states, frames %s" % (a.dst, out["graph"].shape[0], out["observation"].shape[1:]))


if __name__ == "__main__":
    sys.exit(main())

"""vnav — MI355X-native batched cached-scene visual-navigation rollout engine.

Hot path of felipefelixarias/a2cat-vn-pytorch rebuilt for gfx950: the cached-scene
env.step (VectorEnv, libvnav.so) and the A2C rollout/update of the goal-conditioned
CNN policy. See DESIGN.md at the repository root.
"""
from .scenes import (Scene, grid_tables, load_graph_pickle, load_h5, load_npz, maze_scene, oriented_scene,  # noqa: F401
                     oriented_tables, scene_from_arrays, synthetic_scene)
from .envs import CachedThorEnv, VectorEnv, make, to_float_chw  # noqa: F401
from .policy import BigHousePolicy, GoalNavPolicy, PolicyNet  # noqa: F401
from .a2c import A2CTrainer  # noqa: F401
from ._lib import VnavError  # noqa: F401

__version__ = "0.1.0"

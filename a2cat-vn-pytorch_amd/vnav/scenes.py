"""Scene-cache construction on the host (offline; not on the per-step path).

A Scene carries exactly the datasets the cached env reads from its h5 file
(environments/gym_ai2thor/envs/cached.py:26-32): ``graph`` [N,4] int64 (-1 = blocked),
``spd`` (shortest_path_distance) [N,N] int64 and ``observations`` [N,H,W,C] uint8 —
or ``observations=None`` with a ``synth_id`` for frames synthesised on the device.

Builders
  grid_tables(maze)         the h5 writer's row convention, graph/util.py:208-247:
                            state = point*4 + rotation, row = [forward, backward,
                            rot+1, rot-1], spd = cell BFS distance + rotation diff
  synthetic_scene(k)        SURVEY.md §8d synthetic cached-THOR scene: 24x24 grid,
                            Bernoulli(0.3) obstacles at seed 1000+k, largest
                            4-connected component, hash frames
  maze_scene(maze, goal)    graph/env.py SimpleGraphEnv maze as a cached scene
                            (absolute-direction actions, MazeGraph frames)
  oriented_scene(...)       environments/gym_graph/graph.py OrientedGraphEnv over a
                            ThorGridWorld grid (oriented actions, fixed goal list)
  load_graph_pickle(path)   a pickled ThorGridWorld (environments/gym_graph/download.py:
                            37-75) through an allow-list unpickler -> oriented_scene
  scene_from_arrays(...)    h5 datasets already in memory; load_h5 / load_npz read them
                            (tools/h5_to_npz.py converts + optionally resizes offline)
"""
import io
import pickle
from dataclasses import dataclass, field
from typing import Optional, Tuple

import numpy as np
from scipy.sparse import csr_matrix
from scipy.sparse.csgraph import connected_components, shortest_path

DIRECTIONS = ((1, 0), (0, 1), (-1, 0), (0, -1))  # graph/util.py:4-13
CACHED_REWARDS = (1.0, -0.0, 0.0)   # cached.py:84-88: step reward is -reward_configuration[1]
GRAPH_REWARDS = (1.0, 0.0, 0.0)     # graph/env.py rewards=[1.0, 0.0, 0.0]
ORIENTED_REWARDS = (1.0, 0.0, 0.0)  # environments/gym_graph/graph.py:10
_ROT_COST = np.array([0, 1, 2, 1])  # compute_rotation_steps: (r - (gr + d)) % 4 with 3 -> 1


@dataclass
class Scene:
    graph: np.ndarray
    spd: np.ndarray
    frame_shape: Tuple[int, int, int]
    observations: Optional[np.ndarray] = None
    synth_id: int = 0
    rewards: Tuple[float, float, float] = CACHED_REWARDS
    terminal_obs: int = 0  # 0: re-emit previous obs on terminal (cached.py:90-96); 1: current
    # set_complexity semantics: (mode, offset) of vn_set_curriculum. Oriented h5 scenes follow
    # OrientedGraphEnv (uniform over d <= c*(maxd_cell+3)+1; spd carries the rotation term, so
    # maxd_cell + 3 = max spd + 1); maze scenes follow SimpleGraphEnv (0.9/0.1, c*(maxd-1)+1).
    curriculum: Tuple[int, float] = (1, 1.0)
    name: str = ""
    maze: Optional[np.ndarray] = None
    locations: Optional[list] = None
    goals: list = field(default_factory=list)
    # [N,H,W,C] frames emitted as the second output for the current state instead of the goal
    # frame (OrientedGraphEnv's (rgb, third-person rgb) observation)
    companion: Optional[np.ndarray] = None
    # auxiliary observations of GoalGymGraphAuxiliaryEnv (environments/gym_graph/graph.py:96-120):
    # depth [N,H,W,1] and segmentation [N,H,W,3] uint8 per state
    depth: Optional[np.ndarray] = None
    segmentation: Optional[np.ndarray] = None

    @property
    def n_states(self):
        return int(self.graph.shape[0])

    def __post_init__(self):
        self.graph = np.ascontiguousarray(self.graph, dtype=np.int64)
        self.spd = np.ascontiguousarray(self.spd, dtype=np.int64)
        n = self.graph.shape[0]
        if self.graph.shape != (n, 4) or self.spd.shape != (n, n):
            raise ValueError("graph must be [N,4] and spd [N,N]")
        if self.graph.min() < -1 or self.graph.max() >= n:
            raise ValueError("graph entries must lie in [-1, N)")
        if self.observations is not None:
            self.observations = np.ascontiguousarray(self.observations, dtype=np.uint8)
            if self.observations.shape != (n,) + tuple(self.frame_shape):
                raise ValueError("observations must be [N,H,W,C] matching frame_shape")
        if self.companion is not None:
            self.companion = np.ascontiguousarray(self.companion, dtype=np.uint8)
            if self.companion.shape != (n,) + tuple(self.frame_shape):
                raise ValueError("companion frames must be [N,H,W,C] matching frame_shape")
        hw = tuple(self.frame_shape[:2])
        for name, ch in (("depth", 1), ("segmentation", 3)):
            v = getattr(self, name)
            if v is not None:
                v = np.ascontiguousarray(v, dtype=np.uint8)
                if v.ndim == 3:
                    v = v[..., None]
                if v.shape != (n,) + hw + (ch,):
                    raise ValueError("%s must be [N,H,W,%d]" % (name, ch))
                setattr(self, name, v)


def positions(maze):
    """enumerate_positions order (graph/util.py:27-31): row-major over (x, y)."""
    xs, ys = np.nonzero(np.asarray(maze, dtype=bool))
    return list(zip(xs.tolist(), ys.tolist()))


def cell_distances(maze):
    """All-pairs 4-connected BFS distances between free cells, -1 if unreachable."""
    locs = positions(maze)
    lookup = {p: i for i, p in enumerate(locs)}
    rows, cols = [], []
    for i, (x, y) in enumerate(locs):
        for dx, dy in DIRECTIONS:
            j = lookup.get((x + dx, y + dy))
            if j is not None:
                rows.append(i)
                cols.append(j)
    P = len(locs)
    adj = csr_matrix((np.ones(len(rows)), (rows, cols)), shape=(P, P))
    d = shortest_path(adj, method="D", unweighted=True, directed=False)
    out = np.where(np.isinf(d), -1, d).astype(np.int64)
    return out, locs, lookup


def grid_tables(maze):
    """(graph [N,4], spd [N,N], locations) in the h5 writer's convention."""
    base, locs, lookup = cell_distances(maze)
    n = len(locs) * 4
    graph = np.empty((n, 4), dtype=np.int64)
    for p, (x, y) in enumerate(locs):
        for r in range(4):
            fx, fy = DIRECTIONS[r]
            bx, by = DIRECTIONS[(r + 2) % 4]
            f = lookup.get((x + fx, y + fy), -1)
            b = lookup.get((x + bx, y + by), -1)
            graph[p * 4 + r] = (f * 4 + r if f >= 0 else -1, b * 4 + r if b >= 0 else -1,
                                p * 4 + (r + 1) % 4, p * 4 + (r - 1) % 4)
    rot = np.abs(np.arange(4)[:, None] - np.arange(4)[None, :])
    rot[rot == 3] = 1
    spd = (base[:, None, :, None] + rot[None, :, None, :]).reshape(n, n)
    return graph, spd, locs


def synthetic_maze(scene_id, grid=24, obstacle_p=0.3):
    rng = np.random.default_rng(1000 + scene_id)
    free = rng.random((grid, grid)) >= obstacle_p
    adj_rows, adj_cols = [], []
    idx = -np.ones((grid, grid), dtype=np.int64)
    xs, ys = np.nonzero(free)
    idx[xs, ys] = np.arange(len(xs))
    for dx, dy in ((1, 0), (0, 1)):
        a = free[: grid - dx, : grid - dy] & free[dx:, dy:]
        ax, ay = np.nonzero(a)
        adj_rows.append(idx[ax, ay])
        adj_cols.append(idx[ax + dx, ay + dy])
    r = np.concatenate(adj_rows)
    c = np.concatenate(adj_cols)
    m = csr_matrix((np.ones(len(r)), (r, c)), shape=(len(xs), len(xs)))
    _, labels = connected_components(m, directed=False)
    keep = labels == np.bincount(labels).argmax()
    maze = np.zeros((grid, grid), dtype=bool)
    maze[xs[keep], ys[keep]] = True
    return maze


def synthetic_scene(scene_id, grid=24, obstacle_p=0.3, frame_shape=(84, 84, 3)):
    maze = synthetic_maze(scene_id, grid, obstacle_p)
    graph, spd, locs = grid_tables(maze)
    return Scene(graph=graph, spd=spd, frame_shape=tuple(frame_shape), observations=None,
                 synth_id=scene_id, rewards=CACHED_REWARDS, terminal_obs=0,
                 name="synthetic-%d" % scene_id, maze=maze, locations=locs)


def maze_scene(maze, goal, name="maze"):
    """SimpleGraphEnv(MazeGraph(maze, goal)) as a cached scene. Frames are the MazeGraph
    renders (graph/maze_graph.py:20-24) stored as uint8 {0,1}; the policy's u8/255
    input conversion then yields SimpleGraphEnv.observe's render/255 (graph/env.py:110-115)."""
    maze = np.asarray(maze, dtype=bool)
    locs = positions(maze)
    lookup = {p: i for i, p in enumerate(locs)}
    n = len(locs)
    graph = np.full((n, 4), -1, dtype=np.int64)
    for i, (x, y) in enumerate(locs):
        for a, (dx, dy) in enumerate(DIRECTIONS):
            graph[i, a] = lookup.get((x + dx, y + dy), -1)
    base, _, _ = cell_distances(maze)
    X, Y = maze.shape
    frames = np.repeat(maze[None, :, :, None].astype(np.uint8), n, axis=0).repeat(3, axis=3)
    for i, (x, y) in enumerate(locs):
        frames[i, x, y] = (1, 0, 0)
    frames[:, goal[0], goal[1]] = (0, 1, 0)
    g = lookup[tuple(goal)]
    return Scene(graph=graph, spd=base, frame_shape=(X, Y, 3), observations=frames,
                 rewards=GRAPH_REWARDS, terminal_obs=1, name=name, maze=maze, locations=locs,
                 goals=[g], curriculum=(2, -1.0))


def scene_from_arrays(graph, spd, observations, rewards=CACHED_REWARDS, name=""):
    obs = np.asarray(observations, dtype=np.uint8)
    return Scene(graph=graph, spd=spd, frame_shape=tuple(obs.shape[1:]), observations=obs,
                 rewards=rewards, terminal_obs=0, name=name)


def load_npz(path, name=None):
    """A scene converted from a reference h5 file by tools/h5_to_npz.py."""
    d = np.load(path, allow_pickle=False)
    return scene_from_arrays(d["graph"], d["shortest_path_distance"], d["observation"],
                             name=name or path)


def load_h5(path, name=None):
    """A reference h5 scene (graph/util.py:222-227 layout; read as cached.py:26-32). Needs
    h5py; without it convert offline with tools/h5_to_npz.py and use load_npz."""
    try:
        import h5py
    except ImportError as e:
        raise ImportError("h5py is not importable here: convert %s with tools/h5_to_npz.py "
                          "(/opt/conda/bin/python3.9) and load the .npz" % path) from e
    with h5py.File(path, "r") as f:
        return scene_from_arrays(f["graph"][()], f["shortest_path_distance"][()], f["observation"][()],
                                 name=name or path)


def oriented_tables(maze):
    """(graph [N,4], spd [N,N], locations) of OrientedGraphEnv (environments/gym_graph/graph.py:
    9-93) on a grid maze. State = point*4 + rotation over enumerate_positions (graph/util.py:
    27-31). Actions per graph/util.py:15-25: 0 forward along rotation r, 1 rot+1, 2 backward,
    3 rot-1 (rotations are always valid; a move off the free cells is a collision).
    spd[s][g] is the distance sample_initial_state ranks starts by (graph/util.py:119-143):
    cell distance d + compute_rotation_steps (:82-86) where d > 0, 0 on the goal's own cell
    (never a start) and -1 where unreachable."""
    base, locs, lookup = cell_distances(maze)
    P = len(locs)
    n = 4 * P
    nbr = np.full((P, 4), -1, dtype=np.int64)
    for p, (x, y) in enumerate(locs):
        for d, (dx, dy) in enumerate(DIRECTIONS):
            nbr[p, d] = lookup.get((x + dx, y + dy), -1)
    graph = np.empty((n, 4), dtype=np.int64)
    for p in range(P):
        for r in range(4):
            f, b = nbr[p, r], nbr[p, (r + 2) % 4]
            graph[p * 4 + r] = (f * 4 + r if f >= 0 else -1, p * 4 + (r + 1) % 4,
                                b * 4 + r if b >= 0 else -1, p * 4 + (r + 3) % 4)
    # optimal first directions (compute_shortest_path_data, util.py:146-176): the free
    # neighbours one step closer to the goal cell
    rot = np.full((P, P, 4, 4), 99, dtype=np.int64)  # [p, q, r, gr]
    r_idx = np.arange(4)[:, None]
    gr_idx = np.arange(4)[None, :]
    for d in range(4):
        valid = nbr[:, d] >= 0
        nd = np.where(valid[:, None], base[np.maximum(nbr[:, d], 0)], -2)
        opt = valid[:, None] & (nd == base - 1) & (base > 0)
        cost = _ROT_COST[(r_idx - (gr_idx + d)) % 4]
        rot = np.where(opt[:, :, None, None], np.minimum(rot, cost[None, None]), rot)
    spd4 = np.where(base[:, :, None, None] > 0, base[:, :, None, None] + rot,
                    np.where(base[:, :, None, None] == 0, 0, -1))
    spd = spd4.transpose(0, 2, 1, 3).reshape(n, n)
    return graph, np.ascontiguousarray(spd), locs, base


def oriented_scene(maze, observations, goals=(), name="oriented", rewards=ORIENTED_REWARDS,
                   tp_observations=None, depths=None, segmentations=None):
    """OrientedGraphEnv over a ThorGridWorld-style grid. observations [X, Y, 4, H, W, C]
    uint8 indexed (x, y, rotation) as ThorGridWorld.render (graph/thor_graph.py:15-18);
    tp_observations (same shape, optional) are the third-person frames render() appends
    (:26-27), emitted as the second output instead of the goal frame; goals are
    (x, y, rotation) triples (the env's fixed goal list, graph.py:20-23). depths /
    segmentations ([X, Y, 4, H, W, 1|3]) make it GoalGymGraphAuxiliaryEnv's scene
    (graph.py:96-120: rgb, goal rgb, depth, segmentation, goal segmentation).
    Terminal steps emit the current frame (graph.py:86-88); set_complexity follows
    graph.py:51 (opt = c * (largest cell distance + 3) + 1, uniform over the starts)."""
    maze = np.asarray(maze, dtype=bool)
    graph, spd, locs, base = oriented_tables(maze)
    obs = np.asarray(observations)
    if obs.shape[:3] != maze.shape + (4,):
        raise ValueError("observations must be [X, Y, 4, H, W, C] over the maze")
    xs = np.array([p[0] for p in locs])
    ys = np.array([p[1] for p in locs])
    frames = np.ascontiguousarray(obs[xs, ys].reshape((-1,) + obs.shape[3:]), dtype=np.uint8)
    comp = None
    if tp_observations is not None:
        tp = np.asarray(tp_observations)
        if tp.shape != obs.shape:
            raise ValueError("tp_observations must match observations")
        comp = np.ascontiguousarray(tp[xs, ys].reshape((-1,) + tp.shape[3:]), dtype=np.uint8)
    aux = {}
    for key, arr in (("depth", depths), ("segmentation", segmentations)):
        if arr is not None:
            a = np.asarray(arr)
            aux[key] = np.ascontiguousarray(a[xs, ys].reshape((-1,) + a.shape[3:]), dtype=np.uint8)
    lookup = {p: i for i, p in enumerate(locs)}
    goal_states = [lookup[(int(g[0]), int(g[1]))] * 4 + int(g[2]) for g in goals]
    offset = float(base.max() + 3 - spd.max())  # c*(maxd + offset) + 1 == c*(largest + 3) + 1
    return Scene(graph=graph, spd=spd, frame_shape=tuple(frames.shape[1:]), observations=frames,
                 rewards=tuple(rewards), terminal_obs=1, curriculum=(1, offset), name=name, maze=maze,
                 locations=locs, goals=goal_states, companion=comp, **aux)


class _GridWorld:
    """Attribute holder standing in for graph.thor_graph.ThorGridWorld when unpickling."""

    def __setstate__(self, state):
        self.__dict__.update(state)


class _GraphUnpickler(pickle.Unpickler):
    """Allow-list unpickler for ThorGridWorld pickles (graph/util.py:40-79 dump_graph /
    load_graph): only numpy array reconstruction, builtin containers and the grid-world
    class (mapped to a plain attribute holder) resolve — nothing else is importable, so
    loading executes no code from the file."""

    _ALLOWED = {
        ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
        ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
        ("numpy", "ndarray"), ("numpy", "dtype"),
        ("builtins", "tuple"), ("builtins", "list"), ("builtins", "dict"), ("builtins", "set"),
        ("builtins", "frozenset"), ("builtins", "slice"), ("_codecs", "encode"),
    }
    _GRID = {("graph.thor_graph", "ThorGridWorld"), ("graph.core", "GridWorldScene"),
             ("graph.maze_graph", "MazeGraph")}

    def find_class(self, module, name):
        if (module, name) in self._GRID:
            return _GridWorld
        if (module, name) in self._ALLOWED:
            import importlib
            return getattr(importlib.import_module(module), name)
        raise pickle.UnpicklingError("refusing to load %s.%s from a scene pickle" % (module, name))


def load_graph_pickle(path, goals=None, name=None, auxiliary=False):
    """A pickled ThorGridWorld (``~/.visual_navigation/scenes/<name>.pkl``,
    environments/gym_graph/download.py:37-75) as an OrientedGraphEnv scene (or, with
    auxiliary=True, GoalGymGraphAuxiliaryEnv's: goal frame second, depth + segmentation
    attached). goals default to the pickle's own ``goals`` attribute (download.py:11)."""
    with open(path, "rb") as f:
        g = _GraphUnpickler(io.BytesIO(f.read())).load()
    if not isinstance(g, _GridWorld) or "_maze" not in g.__dict__ or "_observations" not in g.__dict__:
        raise ValueError("%s does not hold a ThorGridWorld" % path)
    if goals is None:
        goals = g.__dict__.get("goals") or []
        if isinstance(goals, tuple) and len(goals) == 3 and all(np.isscalar(v) for v in goals):
            goals = [goals]
    if auxiliary:
        return oriented_scene(g._maze, g._observations, goals, name=name or path, depths=g._depths,
                              segmentations=g._segmentations)
    tp = g.__dict__.get("_tp_observations")
    if tp is not None and np.shape(tp) != np.shape(g._observations):
        tp = None  # render() would resize it to the screen size (graph/core.py:29-39): not emitted
    return oriented_scene(g._maze, g._observations, goals, name=name or path, tp_observations=tp)

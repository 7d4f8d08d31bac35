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
  scene_from_arrays(...)    h5 datasets already in memory (see tools/h5_to_npz.py)
"""
from dataclasses import dataclass, field
from typing import Optional, Tuple

import numpy as np
from scipy.sparse import csr_matrix
from scipy.sparse.csgraph import connected_components, shortest_path

DIRECTIONS = ((1, 0), (0, 1), (-1, 0), (0, -1))  # graph/util.py:4-13
CACHED_REWARDS = (1.0, -0.0, 0.0)   # cached.py:84-88: step reward is -reward_configuration[1]
GRAPH_REWARDS = (1.0, 0.0, 0.0)     # graph/env.py rewards=[1.0, 0.0, 0.0]


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

"""Grid-world kernel of graph/util.py restated in numpy (TEST INFRASTRUCTURE ONLY).

Follows, in the reference (felipefelixarias/a2cat-vn-pytorch):
  direction_to_change      graph/util.py:4-13
  step (oriented)          graph/util.py:15-25
  enumerate_positions      graph/util.py:27-31
  is_valid_state           graph/util.py:36-37
  compute_shortest_path_data graph/util.py:146-176 (the recursive DFS relaxation there
                           converges to BFS distances; actions[p,g,d] marks every
                           direction d whose neighbour is one step closer to g)
  save_graph_as_h5 rows    graph/util.py:208-247 (compute_graph_line :212-218, row
                           :231-232, shortest_path_distance :240-247)
"""
from collections import deque

import numpy as np

DIRS = ((1, 0), (0, 1), (-1, 0), (0, -1))


def direction_to_change(direction):
    if direction not in (0, 1, 2, 3):
        raise ValueError("Unsupported direction %s" % direction)
    return DIRS[direction]


def oriented_step(state, action):
    x, y, r = state
    dx, dy = DIRS[r]
    if action == 0:
        return (x + dx, y + dy, r)
    if action == 2:
        return (x - dx, y - dy, r)
    if action == 1:
        return (x, y, (r + 1) % 4)
    if action == 3:
        return (x, y, (r + 3) % 4)
    raise ValueError(action)


def enumerate_positions(maze):
    return [(x, y) for x in range(maze.shape[0]) for y in range(maze.shape[1]) if maze[x, y]]


def is_valid_state(maze, state):
    return (state[0] >= 0 and state[1] >= 0 and state[0] < maze.shape[0]
            and state[1] < maze.shape[1] and bool(maze[state[0], state[1]]))


def shortest_path_data(maze):
    """distances[x,y,gx,gy] int32 (-1 unreachable), actions[x,y,gx,gy,d] bool."""
    X, Y = maze.shape
    distances = np.full((X, Y, X, Y), -1, dtype=np.int32)
    actions = np.zeros((X, Y, X, Y, 4), dtype=bool)
    for gx, gy in enumerate_positions(maze):
        dist = distances[:, :, gx, gy]
        dist[gx, gy] = 0
        q = deque([(gx, gy)])
        while q:
            x, y = q.popleft()
            for dx, dy in DIRS:
                nx, ny = x + dx, y + dy
                if is_valid_state(maze, (nx, ny)) and dist[nx, ny] == -1:
                    dist[nx, ny] = dist[x, y] + 1
                    q.append((nx, ny))
        for x, y in enumerate_positions(maze):
            d = dist[x, y]
            if d <= 0:
                continue
            for k, (dx, dy) in enumerate(DIRS):
                nx, ny = x + dx, y + dy
                if is_valid_state(maze, (nx, ny)) and dist[nx, ny] == d - 1:
                    actions[x, y, gx, gy, k] = True
    return distances, actions


def h5_tables(maze, distances=None):
    """graph [N,4] int64, shortest_path_distance [N,N] int64, location [N,2] f64,
    with state index point*4 + rotation (graph/util.py:208-247)."""
    if distances is None:
        distances, _ = shortest_path_data(maze)
    locations = enumerate_positions(maze)
    lookup = {p: i for i, p in enumerate(locations)}
    n = len(locations) * 4
    graph = np.empty((n, 4), dtype=np.int64)
    location = np.empty((n, 2), dtype=np.float64)
    for point, (x, y) in enumerate(locations):
        for r in range(4):
            fx, fy = DIRS[r]
            bx, by = DIRS[(r + 2) % 4]
            fwd = lookup.get((x + fx, y + fy), -1)
            back = lookup.get((x + bx, y + by), -1)
            graph[point * 4 + r] = [
                -1 if fwd == -1 else fwd * 4 + r,
                -1 if back == -1 else back * 4 + r,
                point * 4 + (r + 1) % 4,
                point * 4 + (r - 1) % 4,
            ]
            location[point * 4 + r] = (x, y)
    P = len(locations)
    xs = np.array([p[0] for p in locations])
    ys = np.array([p[1] for p in locations])
    base = distances[xs[:, None], ys[:, None], xs[None, :], ys[None, :]].astype(np.int64)  # [P,P]
    r = np.arange(4)
    rot = np.abs(r[:, None] - r[None, :])
    rot[rot == 3] = 1
    spd = (base[:, None, :, None] + rot[None, :, None, :]).reshape(n, n)
    return graph, spd, location


def maze_tables(maze, goal):
    """The SimpleGraphEnv maze (graph/env.py:73-143) as a cached scene:
    state = index in enumerate_positions order, action = absolute direction
    (graph/env.py:122), spd[s][g] = BFS distance (util.py:146-176, -1 unreachable)."""
    distances, _ = shortest_path_data(maze)
    locations = enumerate_positions(maze)
    lookup = {p: i for i, p in enumerate(locations)}
    n = len(locations)
    graph = np.full((n, 4), -1, dtype=np.int64)
    for i, (x, y) in enumerate(locations):
        for a, (dx, dy) in enumerate(DIRS):
            graph[i, a] = lookup.get((x + dx, y + dy), -1)
    xs = np.array([p[0] for p in locations])
    ys = np.array([p[1] for p in locations])
    spd = distances[xs[:, None], ys[:, None], xs[None, :], ys[None, :]].astype(np.int64)
    return graph, spd, locations, lookup[tuple(goal)]


def maze_render(maze, state, goal):
    """MazeGraph.render (graph/maze_graph.py:20-24) — float32 [X,Y,3]."""
    render = np.tile(np.expand_dims(maze, 2), [1, 1, 3]).astype(np.float32)
    render[state[0], state[1]] = np.array([1.0, 0.0, 0.0])
    render[goal[0], goal[1]] = np.array([0.0, 1.0, 0.0])
    return render

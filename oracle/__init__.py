"""oracle — CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import anything from here, and only as the checker / the timed CPU baseline. The
product (``a2cat-vn-pytorch_amd/vnav``) never imports it and has no CPU fallback.

Pinning: the restatement is checked against golden vectors produced by running the
reference itself in the build container (``tests/golden/gen_env_goldens.py`` under the
image's Anaconda python3.9 with h5py/skimage, ``tests/golden/gen_model_goldens.py``
under python3.10 + torch) — see ``tests/test_oracle_goldens.py``. The A2C update
math lives in the absent ``deep-rl==0.2.9`` package: that part is "parity unpinned"
(see ``oracle/a2c.py`` and DESIGN.md).

Modules
  philox.py   Philox4x32-10 (the engine's counter RNG contract) in numpy
  graph.py    graph/util.py grid kernel: steps, BFS tables, h5 row builder
  envs.py     cached.py env (single), the batched VectorEnv contract, maze env
  frames.py   synthetic frame hash (scene, state, word) -> uint8 frames
  policy.py   BigGoalHouseModel trunk + heads in torch fp32 (CPU)
  a2c.py      n-step returns / A2C loss / clip / RMSprop restated in torch fp32 (CPU)
"""

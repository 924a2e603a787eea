import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import numpy as np
import oracle as O
from torque_constrained_motion_planning_amd import _lib
from torque_constrained_motion_planning_amd.scene import random_box_scene, obstacle_array
LO = np.array([-2.8973, -1.7628, -2.8973, -3.0718, -2.8973, -0.0175, -2.8973])
HI = np.array([2.8973, 1.7628, 2.8973, -0.0698, 2.8973, 3.7525, 2.8973])
eng = _lib.engine(0)
rng = np.random.default_rng(5)
for n_obs, aligned in ((0, True), (4, True), (16, True), (16, False), (64, True)):
    obs = obstacle_array(random_box_scene(rng, n_obs, aligned=aligned)) if n_obs else np.zeros((0, 15))
    eng.set_scene(obs)
    q = LO + (HI - LO) * rng.random((2000, 7))
    q[:50] = LO - 1e-3 + (HI - LO + 2e-3) * rng.random((50, 7))
    got = eng.collides(q)
    ref = np.array([O.collision(x, obs, cull=2) for x in q])
    bad = np.nonzero(got != ref)[0]
    print(n_obs, aligned, "bad", bad.tolist(), flush=True)
    for i in bad:
        single = eng.collides(q[i:i + 1])[0]
        lim = bool(((q[i] < LO) | (q[i] > HI)).any())
        print("  i", i, "gpu", got[i], "oracle", ref[i], "single", single, "limits", lim,
              "oracle cull0", O.collision(q[i], obs, cull=0), flush=True)
    # repeat the batch: deterministic?
    got2 = eng.collides(q)
    print("  repeat equal", bool((got2 == got).all()), flush=True)
    sub = q[:60]
    eng.set_scene(obs[:8])
    got8 = eng.collides(sub)
    ref8 = np.array([O.collision(x, obs[:8], cull=0) for x in sub])
    print("  obs8 bad", np.nonzero(got8 != ref8)[0].tolist(), flush=True)

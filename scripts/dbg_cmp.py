# temporary (round 4): frames of two library builds compared (RT_LIB_PATH per child), per engine
import os, subprocess, sys, numpy as np
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r"""
import sys, numpy as np
from eraytracer_amd import scenes
from eraytracer_amd.raytracer import render
img = render(640, 480, scenes.named(sys.argv[1]), 3)
np.save(sys.argv[2], img)
"""
for engine in ("fused", "wave"):
    for scene in ("default", "s64"):
        outs = []
        for lib in ("eraytracer_amd/variants/librtmi355x_at_7a588f1.so", ""):
            f = f"/tmp/cmp_{engine}_{scene}_{len(outs)}.npy"
            env = dict(os.environ, RT_ENGINE=engine, RT_LIB_PATH=lib, PYTHONPATH=root)
            r = subprocess.run([sys.executable, "-c", code, scene, f], cwd=root, env=env, capture_output=True, text=True)
            assert r.returncode == 0, r.stderr
            outs.append(np.load(f))
        a, b = outs
        diff = ~np.all(a.view(np.int64) == b.view(np.int64), axis=-1)
        print(engine, scene, "pixels differing between builds:", int(diff.sum()), "max", float(np.abs(a - b).max()), flush=True)
        if diff.sum():
            i = np.argwhere(diff)[0]
            print("  first", i.tolist(), a[tuple(i)].tolist(), b[tuple(i)].tolist())

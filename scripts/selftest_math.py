# rt_selftest_math over many operands: python scripts/selftest_math.py [log2 n] (GPU)
import ctypes, sys, time
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from eraytracer_amd import _native as N
n = 1 << int(sys.argv[1] if len(sys.argv) > 1 else 32)
bad = ctypes.c_uint64(0)
t = time.time()
for seed in (0x5EED, 0xC0FFEE, 0x12345678):
    N.check(N.lib().rt_selftest_math(0, n, seed, ctypes.byref(bad)), "rt_selftest_math")
    print(f"seed {seed:#x}: {n} samples x 4 checks, {bad.value} mismatches ({time.time() - t:.1f} s)", flush=True)
    assert bad.value == 0

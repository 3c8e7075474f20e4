# temporary debugging script (round 4): s256 small frames through the fused path vs the oracle
import ctypes, os, sys, numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eraytracer_amd import _native as N, scenes
from oracle import oracle as O
L = N.lib()
sc = scenes.s256()
el = N.marshal(sc)
st = torch.cuda.current_stream().cuda_stream
def frame(p, w, h, d, spp, fill):
    out = torch.full((L.rt_shard_rows(h, 16, 1), w, 3), fill, dtype=torch.float64, device='cuda')
    N.check(L.rt_launch_spp(p, w, h, d, 16, 0, 1, N.RT_OUT_F64, N.RT_ORDER_EXACT, spp, 5, out.data_ptr(), None, st))
    torch.cuda.synchronize()
    return out.cpu().numpy()[:h]
for (w, h, d, spp) in [(32, 24, 8, 1), (32, 24, 8, 2), (32, 24, 3, 2), (48, 32, 8, 3), (64, 64, 8, 2), (256, 192, 8, 2)]:
    p = ctypes.c_void_p()
    N.check(L.rt_prepare(el, len(el), 0, ctypes.byref(p)))
    N.check(L.rt_configure(p, N.RT_CFG_SIDE_STREAMS, 0))
    ref = O.render(el, w, h, d, mode=O.MEMO, spp=spp, seed=5)
    for rep in range(3):
        img = frame(p, w, h, d, spp, -7.0 - rep)
        err = np.abs(img - ref)
        bad = np.argwhere(err.max(axis=-1) > 1e-5)
        print(os.environ.get("RT_SORT"), w, h, d, spp, "rep", rep, "maxerr", err.max(), "badpx", len(bad), bad[:4].tolist(),
              "stale", int((img == -7.0 - rep).any(axis=-1).sum()), flush=True)
    L.rt_release(p)

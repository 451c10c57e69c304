import time, numpy as np, torch, sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/oracle")
from netstack_amd import Engine, workloads as W
eng = Engine(0)
for n, L in ((1000, 64), (100000, 64), (1000000, 64), (512, 131072)):
    lengths = np.full(n, L, np.uint32)
    flags = np.full(n, 2, np.uint16); flags[0] = 0
    d, end = W.make_desc(lengths, np.zeros(n, np.uint16), align=16, flags=flags)
    arena = torch.randint(0, 256, (end,), dtype=torch.uint8, device="cuda")
    desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    out = eng.batch_tensors(arena, desc, chained=True); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        eng.batch_tensors(arena, desc, out, chained=True)
    torch.cuda.synchronize()
    print(n, L, "one run: %.1f us/launch" % ((time.perf_counter() - t) / 3 * 1e6), flush=True)

import sys, time, numpy as np
sys.path.insert(0, '.')
from flyimg_amd import _lib as L
from flyimg_amd.runtime import Context
from flyimg_amd.processor import ImageProcessor, OptionsBag
rng = np.random.default_rng(20250112)
ops = ["w_300,h_250,c_1", "w_500,smc_1", "w_512,h_512,c_1", "h_300", "w_400,h_400,c_1"]
aspects = [4/3, 3/2, 16/9, 1.0, 2/3, 9/16]
ctx = Context(0)
n = 256
sizes = []
for i in range(n):
    mp = float(np.exp(rng.uniform(np.log(0.5), np.log(24))))
    a = aspects[rng.integers(0, 6)]
    W = max(16, int(round((mp * 1e6 * a) ** 0.5))); H = max(16, int(round(W / a)))
    sizes.append((W, H))
maxb = max(((W * 3 + 15) // 16 * 16) * H for W, H in sizes)
pool = ctx.malloc(maxb)
dst = ctx.malloc(1024 * 1024 * 3 * n)
arr = (L.FiImage * n)()
for i, (W, H) in enumerate(sizes):
    op = ImageProcessor(OptionsBag(ops[i % 5]), W, H).to_op()
    a = arr[i]
    a.src, a.src_w, a.src_h, a.src_stride, a.src_channels = pool, W, H, (W * 3 + 15) // 16 * 16, 3
    a.target_w, a.target_h, a.flags, a.gravity, a.rotate = op.target_w, op.target_h, op.flags, op.gravity, op.rotate
    a.smartcrop_w, a.smartcrop_h = op.smartcrop_w, op.smartcrop_h
    a.dst, a.dst_capacity = dst + i * 1024 * 1024 * 3, 1024 * 1024 * 3
ctx.set_timing(True)
for rep in range(3):
    ctx.reset_stats()
    t = time.perf_counter()
    L.check(ctx.submit_device(arr, n)); L.check(ctx.wait(0))
    el = time.perf_counter() - t
    print(f"rep {rep}: {n} distinct sizes, wall {el*1e3:.1f} ms, host_plan {ctx.stats('host_plan')[0]:.1f} ms, batch {ctx.stats('batch')[0]:.2f} ms, resize {ctx.stats('resize')[0]:.2f} ms",
          {p: ctx.stats(p)[1] for p in ['path_vm','path_fused','path_generic_v','path_generic_h','path_copy']})
    print("status", sum(arr[i].status != 0 for i in range(n)))

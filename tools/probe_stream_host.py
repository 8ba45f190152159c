import sys, time, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import uvhttp_amd as U
eng = U.GpuEngine(0)
n, plen = 65536, 4096
stride = U.gen_frame_stride(plen)
wl = n * stride
wire = torch.empty(wl + 64, dtype=torch.uint8, device="cuda")
eng.gen_frames(wire, n, plen, 7)
conns = n
st = np.zeros(conns, dtype=[("begin", "<u8"), ("len", "<u8"), ("rbs", "<u8"), ("pend", "<u8"), ("pop", "<i4"), ("mf", "<i4"), ("mm", "<i4"), ("srv", "<i4")])
st["begin"] = np.arange(conns, dtype=np.uint64) * stride
st["len"] = stride; st["rbs"] = 65536; st["mf"], st["mm"], st["srv"] = 1 << 24, 1 << 26, 1
sd = torch.from_numpy(st.view(np.uint8).copy()).cuda()
desc = torch.empty(n * 32, dtype=torch.uint8, device="cuda"); res = torch.empty(conns * 64, dtype=torch.uint8, device="cuda")
for timing in (False, True):
    eng.set_timing(timing)
    for k in range(3):
        torch.cuda.synchronize()
        ts = []
        for i in range(20):
            t0 = time.perf_counter()
            eng.decode_streams(wire, sd, conns, n, desc=desc, results=res, wire_len=wl)
            ts.append(time.perf_counter() - t0)
        t1 = time.perf_counter(); torch.cuda.synchronize(); t2 = time.perf_counter()
        print("timing", timing, "host per call us", [round(x * 1e6) for x in ts[:5]], "median", round(sorted(ts)[10] * 1e6), "drain", round((t2 - t1) * 1e6))
    eng.kernel_time()

#!/usr/bin/env python3
"""Device stamps against HIP events on the same calls (why the stamped C3 payload kernel read
2-3 % above the bench step).

  python tools/stamp_probe.py [c3] [c2] ...

For each config: K calls back to back between two events (stamps on), then the stamp timeline
of those calls.  Reports the events' per-call time, the stamped chain (first kernel's begin to
the last kernel's end) per call, and the ratio of the stamped span of all K calls (first begin
to last end) to the events' span — a clock-rate error shows as that ratio != 1 on every config,
a late / early stamp word as a per-call chain above the per-call event time.  The rows differ in
what precedes the measured calls: nothing, an idle host pause, or the clearing read_stamps()
(a 71 MB copy back) with and without warm-up calls after it — the device's clocks after an idle."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import uvhttp_amd as U  # noqa: E402

CFG = {"c2": (65536, 4096), "c3": (65536, 65536), "c4": (1048576, 256)}


def main():
    K = 12
    for cfg in sys.argv[1:] or ["c3", "c2"]:
        n, plen = CFG[cfg]
        e = U.GpuEngine(0)
        stride = U.gen_frame_stride(plen)
        wl = stride * n
        wire = torch.empty(wl + 64, dtype=torch.uint8, device="cuda")
        e.gen_frames(wire, n, plen, 7, opcode0=2)
        desc, summ = e.alloc_outputs(n)
        for _ in range(3):
            e.decode_inplace(wire, n, stride=stride, wire_len=wl, desc=desc, summary=summ)
        torch.cuda.synchronize()
        # (stamps, idle before the measured calls, warm-up calls after the idle / the clear)
        for stamps, idle, warm in ((False, 0, 0), (False, 0.05, 0), (True, 0, 0), (True, 0, 40),
                                   (False, 0, 0)):
            e.set_stamps(stamps)
            e.read_stamps() if stamps else None
            time.sleep(idle)
            for _ in range(warm):
                e.decode_inplace(wire, n, stride=stride, wire_len=wl, desc=desc, summary=summ)
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
            evs[0].record()
            for k in range(K):
                e.decode_inplace(wire, n, stride=stride, wire_len=wl, desc=desc, summary=summ)
                evs[k + 1].record()
            torch.cuda.synchronize()
            per = [evs[k].elapsed_time(evs[k + 1]) * 1000 for k in range(1, K)]  # (first: launch)
            span_ev = evs[1].elapsed_time(evs[K]) * 1000
            line = f"{cfg} stamps={int(stamps)} idle={idle} warm={warm:2d} event per call median {statistics.median(per):8.1f} us"
            if stamps:
                recs = e.read_stamps()
                calls = sorted({r[0] for r in recs})[-K:]
                by = {c: [r for r in recs if r[0] == c] for c in calls}
                chain = [(max(r[3] for r in by[c]) - min(r[2] for r in by[c])) / 1000 for c in calls]
                pay = [(r[3] - r[2]) / 1000 for c in calls for r in by[c] if r[1] == "payload"]
                ends = [max(r[3] for r in by[c]) for c in calls]
                span_st = (ends[-1] - ends[0]) / 1000  # end of call 1 .. end of call K-1 (as span_ev)
                line += (f" | stamped chain median {statistics.median(chain):8.1f} payload "
                         f"{statistics.median(pay):8.1f} us | span stamps/events "
                         f"{span_st:9.1f}/{span_ev:9.1f} = {span_st / span_ev:.4f}")
                gaps = [(min(r[2] for r in by[calls[i + 1]]) - ends[i]) / 1000 for i in range(len(calls) - 1)]
                line += f" | gap between calls median {statistics.median(gaps):6.2f} min {min(gaps):6.2f} us"
            print(line, flush=True)
        e.close()


if __name__ == "__main__":
    main()

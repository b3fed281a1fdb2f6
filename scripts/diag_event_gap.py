"""Cost of a cross-stream fork on the PRODUCER stream: the gap between two back-to-back kernels
on one stream when an event is recorded between them (and another stream waits on it), by event
flavour.  Run under ``rocprofv3 --kernel-trace`` and read the gaps with ``--analyze``:

    rocprofv3 --kernel-trace -d gpurun_out/evgap -- python scripts/diag_event_gap.py
    python scripts/diag_event_gap.py --analyze gpurun_out/evgap/.../kernel_trace.csv

Phases (separated by a host sleep, so the trace splits them by time): plain back-to-back,
torch event (hipEventDisableTiming), + hipEventDisableSystemFence, + hipEventReleaseToDevice,
hipStreamWriteValue64 / WaitValue64 hand-off."""
import ctypes
import sys
import time

PHASES = ["plain", "torch_event", "nofence", "release_device", "write_value"]
REPS = 40


def run():
    import torch
    hip = ctypes.CDLL("libamdhip64.so")
    dev = torch.device("cuda:0")
    x = torch.ones(16 << 20, device=dev, dtype=torch.float32)  # 64 MB: ~25 us per pass
    y = torch.ones(1 << 16, device=dev)
    side = torch.cuda.Stream(device=dev)
    main = torch.cuda.current_stream(dev)

    def mk(flags):
        ev = ctypes.c_void_p()
        assert hip.hipEventCreateWithFlags(ctypes.byref(ev), ctypes.c_uint(flags)) == 0
        return ev

    evs = {"nofence": mk(0x2 | 0x20000000), "release_device": mk(0x2 | 0x40000000)}
    sig = ctypes.c_void_p()
    assert hip.hipExtMallocWithFlags(ctypes.byref(sig), ctypes.c_size_t(8), ctypes.c_uint(0x2)) == 0
    assert hip.hipMemset(sig, 0, ctypes.c_size_t(8)) == 0
    torch.cuda.synchronize()
    ticket = [0]
    ms, ss = ctypes.c_void_p(main.cuda_stream), ctypes.c_void_p(side.cuda_stream)
    for phase in PHASES:
        for _ in range(REPS):
            x.mul_(1.0)
            if phase == "torch_event":
                side.wait_stream(main)
            elif phase in evs:
                assert hip.hipEventRecord(evs[phase], ms) == 0
                assert hip.hipStreamWaitEvent(ss, evs[phase], ctypes.c_uint(0)) == 0
            elif phase == "write_value":
                ticket[0] += 1
                assert hip.hipStreamWriteValue64(ms, sig, ctypes.c_uint64(ticket[0]), ctypes.c_uint(0)) == 0
                assert hip.hipStreamWaitValue64(ss, sig, ctypes.c_uint64(ticket[0]), ctypes.c_uint(0),
                                                ctypes.c_uint64(~0 & 0xFFFFFFFFFFFFFFFF)) == 0
            if phase != "plain":
                with torch.cuda.stream(side):
                    y.add_(1.0)
            x.mul_(1.0)
        torch.cuda.synchronize()
        time.sleep(0.02)
    print("ok", flush=True)


def analyze_wake(path):
    """evgap.hip's last phase: main-stream pass start minus the end of the side stream's last pass"""
    import csv
    rows = sorted((r for r in csv.DictReader(open(path)) if "big_pass" in r["Kernel_Name"]),
                  key=lambda r: int(r["Start_Timestamp"]))
    side = [r for r in rows if int(r["Grid_Size_X"]) and r["Stream_Id"] != rows[0]["Stream_Id"]]
    main_after = [r for r in rows if r["Stream_Id"] == rows[0]["Stream_Id"]][-40:]
    lat = []
    for m in main_after:
        ends = [int(s["End_Timestamp"]) for s in side if int(s["End_Timestamp"]) <= int(m["Start_Timestamp"])]
        if ends:
            lat.append((int(m["Start_Timestamp"]) - max(ends)) / 1000)
    lat.sort()
    print(f"wake            n {len(lat):3d}  latency median {lat[len(lat) // 2]:6.2f} us  p90 {lat[int(len(lat) * 0.9)]:6.2f}")


def analyze(path, names=PHASES, key="elementwise", skip_last=0):
    import csv
    rows = [r for r in csv.DictReader(open(path)) if key in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    big = [r for r in rows if key != "elementwise" or int(r["Grid_Size_X"]) > (1 << 20)]  # the 64 MB passes (main stream)
    phases, cur = [], [big[0]]
    for a, b in zip(big, big[1:]):
        if int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) > 5_000_000:  # > 5 ms: next phase
            phases.append(cur)
            cur = []
        cur.append(b)
    phases.append(cur)
    # a phase's first fork may stall on first-use setup (stream creation): drop runts, and the odd
    # leading kernel of a phase split by such a stall
    phases = [ph[len(ph) % 2:] for ph in phases if len(ph) >= 4]
    if skip_last:
        phases = phases[:-skip_last]
    for name, ph in zip(names, phases[-len(names):]):
        gaps = sorted((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1000
                      for a, b in zip(ph[0::2], ph[1::2]))
        dur = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in ph)
        print(f"{name:15s} pairs {len(gaps):3d}  gap median {gaps[len(gaps) // 2]:6.2f} us  "
              f"p90 {gaps[int(len(gaps) * 0.9)]:6.2f}  kernel median {dur[len(dur) // 2]:6.2f} us")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    elif len(sys.argv) > 2 and sys.argv[1] == "--analyze-bin":  # scripts/evgap.hip
        names = ["plain", "marker", "bound", "rec_only", "side_only", "rec_wait", "wait_done"]
        analyze_wake(sys.argv[2])
        analyze(sys.argv[2], names, "big_pass", skip_last=1)
    else:
        run()

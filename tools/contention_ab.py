"""Diagnostic: the C2 frame while other kernels hold some CUs -- what the multi-GPU step sees
when RCCL's all-gather kernels (one workgroup per channel, on their own stream) run beside the
next frame's render.  Each frame, n_occ single-wave spin kernels (torch.cuda._sleep, each on
its own stream, so they run concurrently) are launched just before the frame; a resident wave
keeps the tile kernel's 512-thread, 256-VGPR workgroup off its CU for the spin's duration.

Reports the frame time (host clock around K frames, synchronised) for n_occ = 0 and the given
counts, and the spin length used.  usage: contention_ab.py [--occ=0/8/16/32] [--spin-us=600]
"""
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402


def main():
    occ = [0, 8, 16, 32]
    spin_us = 600.0
    for a in sys.argv[1:]:
        if a.startswith("--occ="):
            occ = [int(x) for x in a[6:].replace("/", ",").split(",")]
        elif a.startswith("--spin-us="):
            spin_us = float(a[10:])
    dev = torch.device("cuda:0")
    from scenedino_amd import _lib
    _lib.load()
    net, renderer, wrapper, sampler, pose, Ks = bench.make_scene(0, dev, "bf16", offset_pose=True)
    # calibrate _sleep cycles -> us
    s = torch.cuda.Stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        e0.record()
        torch.cuda._sleep(1_000_000)
        e1.record()
    torch.cuda.synchronize()
    cyc_per_us = 1_000_000 / (e0.elapsed_time(e1) * 1e3)
    cycles = int(spin_us * cyc_per_us)
    streams = [torch.cuda.Stream() for _ in range(max(occ))]
    main_s = torch.cuda.current_stream()
    print(f"spin {spin_us:.0f} us = {cycles} cycles; offset pose, bf16", flush=True)

    def frame(n):
        if n:
            ev = torch.cuda.Event()
            ev.record(main_s)
            for st in streams[:n]:
                st.wait_event(ev)
                with torch.cuda.stream(st):
                    torch.cuda._sleep(cycles)
        bench.render_step(net, wrapper, sampler, pose, Ks)

    with torch.no_grad():
        for n in occ:
            for _ in range(5):
                frame(n)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            steps = 20
            for _ in range(steps):
                frame(n)
            torch.cuda.synchronize()
            # the spins of the last frame may outlast it: wait for them too
            dt = (time.perf_counter() - t0) / steps
            print(f"occupied waves {n:3d}: {dt * 1e3:.3f} ms per frame (render + spins overlapped)",
                  flush=True)


if __name__ == "__main__":
    main()

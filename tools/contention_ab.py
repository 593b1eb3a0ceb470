"""Diagnostic: the C2 frame while another kernel holds some CUs -- what the multi-GPU step sees
when RCCL's all-gather of the previous frame (one workgroup per channel, its own stream) runs
beside the next frame's projection and render.  Each frame, ONE kernel of n_occ single-wave
workgroups (sd_spin, on a side stream; its workgroups spread over the XCDs like RCCL's) is
launched just before the frame; a resident wave keeps a 512-thread, 256-VGPR persistent
workgroup off its CU for the spin's duration.  --reserve=R: the library's persistent grids
leave R CUs free (sd_reserve_cus), as bench.py does for the RCCL gather.

Reports the frame time (host clock around 20 frames, synchronised) per n_occ.
usage: contention_ab.py [--occ=0/8/16/32] [--spin-us=600] [--reserve=0]
"""
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402


def main():
    occ = [0, 8, 16, 32]
    spin_us = 600.0
    reserve = 0
    for a in sys.argv[1:]:
        if a.startswith("--occ="):
            occ = [int(x) for x in a[6:].replace("/", ",").split(",")]
        elif a.startswith("--spin-us="):
            spin_us = float(a[10:])
        elif a.startswith("--reserve="):
            reserve = int(a[10:])
    dev = torch.device("cuda:0")
    from scenedino_amd import _lib
    _lib.load()
    _lib.reserve_cus(reserve)
    net, renderer, wrapper, sampler, pose, Ks = bench.make_scene(0, dev, "bf16", offset_pose=True)
    side = torch.cuda.Stream()
    main_s = torch.cuda.current_stream()
    print(f"spin {spin_us:.0f} us; reserved CUs {reserve}; offset pose, bf16", flush=True)

    def frame(n):
        if n:
            ev = torch.cuda.Event()
            ev.record(main_s)
            side.wait_event(ev)
            _lib.spin(n, spin_us, side)
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

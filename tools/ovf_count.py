"""Diagnostic: how many rays of a C1 / C2 frame the tile kernel sends to its overflow list
(groups whose tap box does not fit a tile buffer; rendered by the per-ray k_render_proj).
usage: ovf_count.py [--k=32] [--identity]"""
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402


def main():
    offset = "--identity" not in sys.argv
    for a in sys.argv[1:]:
        if a.startswith("--k="):
            bench.K_SAMPLES = int(a[4:])
    dev = torch.device("cuda:0")
    net, renderer, wrapper, sampler, pose, Ks = bench.make_scene(0, dev, "bf16", offset)
    with torch.no_grad():
        bench.render_step(net, wrapper, sampler, pose, Ks)
        torch.cuda.synchronize()
    work = net._last_render_work.view(torch.int32)
    R = bench.H * bench.W
    # per-workgroup lists at the end of work (sdhip_render.h): [ncu] counts, [ncu][cap] blocks
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    cap = ((R + ncu - 1) // ncu + 64) // 4 + 1
    list_words = ((4 * (ncu + ncu * cap) + 15) // 16) * 16 // 4
    ovf = work[work.numel() - list_words:]
    nblk = int(ovf[:ncu].sum().item())
    print(f"{'offset' if offset else 'identity'} K={bench.K_SAMPLES}: {nblk} overflow 4-ray blocks = "
          f"{4 * nblk} rays of {R} ({100.0 * 4 * nblk / R:.2f} %)")


if __name__ == "__main__":
    main()

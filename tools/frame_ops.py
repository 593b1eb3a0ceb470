"""Diagnostic: the torch ops issued per C2 frame besides the libsdhip.so kernels
(torch.profiler, 10 frames at the offset pose), with the Python call site of each."""
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, ".")
import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    net, renderer, wrapper, sampler, pose, Ks = bench.make_scene(0, dev, "bf16", True)
    with torch.no_grad():
        for _ in range(3):
            bench.render_step(net, wrapper, sampler, pose, Ks)
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
            for _ in range(10):
                bench.render_step(net, wrapper, sampler, pose, Ks)
            torch.cuda.synchronize()
    print(prof.key_averages(group_by_stack_n=6).table(sort_by="count", row_limit=40,
                                                      max_name_column_width=40))


main()

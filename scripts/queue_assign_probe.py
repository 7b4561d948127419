#!/usr/bin/env python3
"""Which hardware queue each torch stream lands on, in creation order (run under
`rocprofv3 --kernel-trace`, then scripts/queue_map.py on the trace). The process mirrors the
data-parallel step's stream set-up: the high-priority main stream first (parallel/engine.py
use_priority_main_stream), then normal-priority streams as the executor (weight-gradient side
stream), the report stream, the process group and a feeder would take them. Stream k runs k+1
tiny kernels so the trace's stream ids can be matched to creation order.

    rocprofv3 --kernel-trace -d out -o tr --output-format csv -- python3 scripts/queue_assign_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    from distributed_resnet_tensorflow_amd.parallel.engine import use_priority_main_stream
    use_priority_main_stream()
    main_s = torch.cuda.current_stream()
    x = torch.zeros(1024, device="cuda")
    x.add_(1)
    streams = [torch.cuda.Stream() for _ in range(n)]
    for k, s in enumerate(streams):
        with torch.cuda.stream(s):
            for _ in range(k + 2):
                x.add_(1)
    torch.cuda.synchronize()
    print("main", hex(main_s.cuda_stream))
    for k, s in enumerate(streams):
        print(f"normal stream {k}: {k + 2} kernels, handle {hex(s.cuda_stream)}")


if __name__ == "__main__":
    main()

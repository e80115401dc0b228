"""HIP graph capture of launch-bound steps.

At small batches (BASELINE C2: one 2048^2 slice) a MED-PEE embed + extract is ~25 us of GPU
work, and the host path (Python -> ctypes -> C ABI -> hipLaunchKernel) is of the same order
(under rocprofv3's tracing the GPU idles 4-7 us before each launch, tools/archive/c2_prof.sh).
Eagerly the step is two launches: small out-of-place batches run the self-cleaning look-back
passes, whose call epoch the library counts on the host (round 5).  A captured call cannot
take that path -- every replay would repeat the captured epoch -- so the library gives a
call made under stream capture the zeroing variant instead: the captured step is four
launches (a zeroing launch before each look-back pass), and every replay starts from clean
status words.  torch.cuda.CUDAGraph drives hipStreamBeginCapture on its capture stream,
which is the current stream our C ABI launches on; replaying issues the launches with one
host call.  Valid because every launch path of the library is capture-safe: no allocation,
no host synchronisation, no memcpy to the host; all state lives in the caller's buffers,
which the replay reuses (same device pointers, so the inputs are refreshed in place between
replays, not re-bound).

Measured at C2 (bench.py --c2-graph 1): the replayed step takes 0.0307 ms against 0.0242 ms
for the eager loop, whose launches already run ahead of the GPU -- the graph launch costs
more than it saves here, so the bench and the codecs launch eagerly.  What this module keeps
is the property, tested on the GPU (tests/test_pee.py::test_gpu_pee_step_graph_replay): a
caller that embeds the codec in its own captured pipeline gets exact results on replay.
"""
from __future__ import annotations


def capture(fn, warmup: int = 2):
    """Run fn() `warmup` times on a side stream (first-call work: the per-device CU count,
    lazy HIP module loads), then capture one call into a graph; returns the
    torch.cuda.CUDAGraph (replay() re-issues exactly those launches on the current stream)."""
    import torch
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(warmup):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    torch.cuda.synchronize()
    return g

"""hipGraph capture of repeated kernel evaluations (torch.cuda.CUDAGraph is a hipGraph on ROCm).

The C ABI (include/gpsig_amd.h) never allocates and never synchronises the host, and every launch
is ordered on the caller's stream, so a whole K(X) evaluation -- feature records, diagonal, Gram
kernel, fused normalisation -- can be captured once and replayed: the per-call host work (argument
checks, ctypes, torch launches) disappears, which is what bounds small problems (the reference's
C1-sized calls, minibatch kernels inside a training loop).  Inputs are copied into static buffers
before each replay; shapes are fixed by the capture.

    kern.to("cuda")                                  # hyperparameters on the device: no H2D copies
    gram = GraphedCall(lambda X: kern.K(X), X0)
    K = gram(X1)        # same as kern.K(X1), replayed from the graph

Forward evaluation only (no autograd through a replay).
"""
from __future__ import annotations

import torch


class GraphedCall:
    """Capture fn(*inputs) (device tensors in, device tensor(s) out) into a graph on the current
    device; calling the object copies new inputs into the captured buffers and replays."""

    def __init__(self, fn, *example_inputs, warmup: int = 2):
        for x in example_inputs:
            if not (isinstance(x, torch.Tensor) and x.is_cuda):
                raise ValueError("graph capture needs device tensors as inputs")
        self.fn = fn
        self.static_in = [x.detach().clone() for x in example_inputs]
        self.stream = torch.cuda.Stream()
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.no_grad(), torch.cuda.stream(self.stream):
            # warm-up on the capture stream: sizes the per-stream workspace (gpsig_amd.ops.workspace)
            # and loads the library before capture
            for _ in range(warmup):
                fn(*self.static_in)
        torch.cuda.current_stream().wait_stream(self.stream)
        self.graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(self.graph, stream=self.stream):
            self.static_out = fn(*self.static_in)
        # the captured launches address this capture stream's scratch buffer: hold it for the graph's
        # lifetime (gpsig_amd.ops.release_workspaces() only drops the cache's references); other
        # streams' buffers stay releasable
        from . import ops
        key = (torch.cuda.current_device() if example_inputs[0].device.index is None
               else example_inputs[0].device.index, self.stream.cuda_stream)
        with ops._ws_lock:
            self._scratch = ops._ws.get(key)

    def __call__(self, *inputs):
        if len(inputs) != len(self.static_in):
            raise ValueError(f"expected {len(self.static_in)} inputs")
        for s, x in zip(self.static_in, inputs):
            if x.shape != s.shape:
                raise ValueError(f"input shape {tuple(x.shape)} differs from the captured {tuple(s.shape)}")
            s.copy_(x)
        self.graph.replay()
        return self.static_out

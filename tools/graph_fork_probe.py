"""Does a hipGraph captured with a fork/join over two streams run its branches concurrently?
Two independent chains of GEMMs (each sized to occupy only part of the GPU) are captured
(a) on one stream and (b) forked onto two streams; prints replay times of both graphs and
of each chain alone.  A concurrent graph replays in ~max(chain), a serial one in ~sum."""
import json
import torch


def main():
    dev = "cuda"
    a = torch.randn(2048, 2048, device=dev, dtype=torch.bfloat16)
    b = torch.randn(2048, 2048, device=dev, dtype=torch.bfloat16)
    x = torch.randn(64, 4096, device=dev, dtype=torch.float32)
    outs = [torch.empty(2048, 2048, device=dev, dtype=torch.bfloat16) for _ in range(2)]
    xo = torch.empty_like(x)

    def chain_a():
        for _ in range(40):
            torch.mm(a, b, out=outs[0])

    def chain_b():
        for _ in range(400):
            torch.tanh(x, out=xo)

    side = torch.cuda.Stream()

    def forked():
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            chain_b()
        chain_a()
        torch.cuda.current_stream().wait_stream(side)

    def serial():
        chain_a()
        chain_b()

    res = {}
    for name, fn in (("a", chain_a), ("b", chain_b), ("serial", serial), ("forked", forked)):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) / 10, 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

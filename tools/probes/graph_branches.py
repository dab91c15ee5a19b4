"""Do forked streams captured into one HIP graph run concurrently on replay?  Two 1-wave spin kernels
(torch.cuda._sleep) in sequence vs on two forked streams; prints both replay times.
    python tools/probes/graph_branches.py"""
import torch


def timed(g, n=20):
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    cyc = 2_000_000
    torch.cuda._sleep(cyc)
    torch.cuda.synchronize()
    seq = torch.cuda.CUDAGraph()
    with torch.cuda.graph(seq):
        torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)
    par = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    with torch.cuda.graph(par):
        main_s = torch.cuda.current_stream()
        side.wait_stream(main_s)
        torch.cuda._sleep(cyc)
        with torch.cuda.stream(side):
            torch.cuda._sleep(cyc)
        main_s.wait_stream(side)
    one = torch.cuda.CUDAGraph()
    with torch.cuda.graph(one):
        torch.cuda._sleep(cyc)
    print(f"one sleep {timed(one):.3f} ms | two in sequence {timed(seq):.3f} ms | two forked {timed(par):.3f} ms",
          flush=True)


if __name__ == "__main__":
    main()

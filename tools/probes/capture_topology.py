"""Which graph-capture stream topology crashes hipStreamEndCapture?  Patterns of the pipelined
mapping iteration with trivial torch ops, simplest first; each prints before and after its
capture (a segfault ends the process at the first failing pattern)."""
import sys

import torch

dev = torch.device("cuda:0")
x = torch.zeros(1 << 20, device=dev)
sc, sf, sg = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()


def t1():  # fork sc, join only in the tail
    main = torch.cuda.current_stream()
    x.add_(1)
    sc.wait_stream(main)
    with torch.cuda.stream(sc):
        x.mul_(1.0)


def t2():  # + a tensor allocated on main in capture, used on sc, record_stream, freed before the end
    main = torch.cuda.current_stream()
    y = torch.empty(1 << 16, device=dev)
    y.fill_(2)
    sc.wait_stream(main)
    y.record_stream(sc)
    with torch.cuda.stream(sc):
        x[: 1 << 16].add_(y)
    del y


def t3():  # + nested fork sg off sc, sc waits sg
    t2()
    sg.wait_stream(sc)
    with torch.cuda.stream(sg):
        x.add_(3)
    with torch.cuda.stream(sc):
        x.add_(4)
    sc.wait_stream(sg)


def t4():  # + a second branch sf joined inside fn
    main = torch.cuda.current_stream()
    t3()
    sf.wait_stream(main)
    with torch.cuda.stream(sf):
        x.add_(5)
    main.wait_stream(sf)


def t5():  # + sc forked and joined earlier in the same fn (the forward half)
    main = torch.cuda.current_stream()
    sc.wait_stream(main)
    with torch.cuda.stream(sc):
        x.add_(6)
    main.wait_stream(sc)
    t4()


def tail():
    torch.cuda.current_stream().wait_stream(sc)


def c2():  # candidate: sf (forked from main) also waits on sc mid-way, then joins main; sc joins in the tail
    main = torch.cuda.current_stream()
    sc.wait_stream(main)
    sf.wait_stream(main)
    with torch.cuda.stream(sc):
        x.add_(1)            # lean
    with torch.cuda.stream(sf):
        x[:16].add_(2)       # frozen branch
    sf.wait_stream(sc)
    with torch.cuda.stream(sf):
        x[16:32].add_(3)     # colour grid adam
    with torch.cuda.stream(sc):
        x[32:64].add_(4)     # wgrad
    main.wait_stream(sf)


def c3():  # c2 with the forward half forked and joined first
    main = torch.cuda.current_stream()
    sc.wait_stream(main)
    with torch.cuda.stream(sc):
        x.add_(6)
    main.wait_stream(sc)
    c2()


ORDER = [("t1", t1), ("t2", t2), ("c2", c2), ("c3", c3), ("t4", t4), ("t3", t3), ("t5", t5)]
if len(sys.argv) > 1:
    ORDER = [(n, f) for n, f in ORDER if n in sys.argv[1:]]
for name, fn in ORDER:
    for _ in range(2):  # eager warm-up like StepGraphs
        fn()
        tail()
    torch.cuda.synchronize()
    print(name, "capture ...", flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
        tail()
    g.replay()
    torch.cuda.synchronize()
    print(name, "ok", flush=True)
    g2 = torch.cuda.CUDAGraph()  # a block of 3 iterations, one tail
    with torch.cuda.graph(g2):
        for _ in range(3):
            fn()
        tail()
    g2.replay()
    torch.cuda.synchronize()
    print(name, "block ok", flush=True)
sys.exit(0)

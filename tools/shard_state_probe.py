"""Does a 125k-pair S2 shard's fp32 pass depend on what the process did before?
Per-run fp32 kernel times of rank 0's 1/8 shard: in a fresh process, while the
full 1M-pair batch is resident, after it is freed, and after a flat call."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gatk-haplotypecaller-cpp17_amd"))
import hcphmm  # noqa: E402
import shard  # noqa: E402
import workloads as W  # noqa: E402

hcphmm.init(0)
b = W.config("S2")
sh = W.subset(b, shard.shard_pairs(b["R"], b["H"], 8)[0])


def measure(label, warm=5, n=10):
    bb = hcphmm.Batch(sh)
    for _ in range(warm):
        bb.run()
    bb.stats()
    t = []
    for _ in range(n):
        bb.run()
        t.append(round(bb.stats().kernel_ms_f32, 4))
    bb.close()
    print(label, "median", sorted(t)[len(t) // 2], t, flush=True)


measure("fresh process")
measure("fresh process, again")
big = hcphmm.Batch(b)
big.run()
big.stats()
measure("1M batch resident")
big.close()
measure("1M batch freed")
hcphmm.pairs(b)
measure("after a flat 1M call")

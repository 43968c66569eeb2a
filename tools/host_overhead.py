"""Where does a build step's wall time go?  Host return time of each call vs
device time (diagnostic)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs265-lsm-tree_amd"))
import torch
import bloomhip as bh

keys = torch.from_numpy(bh.gen_puts(13141, 16_777_216)).cuda()
m = bh.m_bits(16_777_216, 10.0)
f = bh.BloomFilter(m)
s = torch.cuda.current_stream()
print("torch stream handle", s.cuda_stream, "lib stream", f.stream_ptr())
for _ in range(3):
    f.clear(stream=s); f.set_batch(keys, stream=s)
torch.cuda.synchronize()

def run(label, fn, K=50):
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(K):
        a = time.perf_counter(); fn(); host.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{label:28s} wall/step {1e6*(t2-t0)/K:8.1f} us  host-return/step {1e6*sum(host)/K:8.1f} us  (max {1e6*max(host):.1f})")

run("clear+set (torch stream)", lambda: (f.clear(stream=s), f.set_batch(keys, stream=s)))
run("set only", lambda: f.set_batch(keys, stream=s))
run("clear only", lambda: f.clear(stream=s))
ls = f.stream_ptr()
run("clear+set (lib stream)", lambda: (f.clear(stream=ls), f.set_batch(keys, stream=ls)))
side = torch.cuda.Stream()
run("clear+set (side stream)", lambda: (f.clear(stream=side), f.set_batch(keys, stream=side)))
f.set_strategy(bh.BUILD_ATOMIC)
run("atomic build", lambda: f.set_batch(keys, stream=s), K=5)

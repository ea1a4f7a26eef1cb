"""PMC workloads (dev tool):
python tools/kern_workloads.py {inverse M BATCH | group N M COUNT | grams N M COUNT | pc N M COUNT | pcg M COUNT} [reps]
inverse: engine.hessian_inverse_batched on BATCH synthetic Grams of order M (N = 262144 scale);
group:   pt2q_quantize_blocks_group of COUNT fp16 N x M linears (SSR, variant M);
pc:      per-channel block loops (block_size = M, config C5) of COUNT bf16 N x M linears;
grams:   engine.gram_batched over COUNT Grams of DISTINCT (env, default 4) resident fp16 N x M
         activations rotated over the items (as the bench)."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pt2q_loader
pt2q = pt2q_loader.load()
kind = sys.argv[1]
reps = int(sys.argv[5]) if len(sys.argv) > 5 and sys.argv[1] != "pcg" else (int(sys.argv[4]) if sys.argv[1] == "pcg" and len(sys.argv) > 4 else 3)
if kind == "inverse":
    m, batch = int(sys.argv[2]), int(sys.argv[3])
    X = pt2q.fill_synthetic((4 * m, m), 77, outliers=True).half()
    G1 = pt2q.gram(X)
    G = G1.expand(batch, m, m).contiguous()
    for _ in range(reps):
        Hinv, info = pt2q.engine.hessian_inverse_batched(G, 4 * m, chunk=batch)
    torch.cuda.synchronize()
    print("inverse done", int(info.max()))
elif kind == "grams":
    # DISTINCT (env, default 4) activation tensors rotated over the items, as bench.py's step
    n, m, count = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    nd = int(os.environ.get("DISTINCT", "4"))
    Xs = [pt2q.fill_synthetic((n, m), 79 + 7919 * k, outliers=True).half() for k in range(nd)]
    G = torch.empty(count, m, m, device=Xs[0].device)
    for _ in range(reps):
        pt2q.engine.gram_batched([Xs[z % nd] for z in range(count)], G)
    torch.cuda.synchronize()
    print("grams done", float(G[0, 0, 0]))
elif kind == "pcg":  # grouped per-channel rows (C5's q/k/v/o and gate/up row counts): pcg M COUNT
    m, count = int(sys.argv[2]), int(sys.argv[3])
    X = pt2q.fill_synthetic((4096, m), 78, outliers=True).bfloat16()
    G = pt2q.gram(X)
    S1d = pt2q.engine.s1_from_gram_batched(G.unsqueeze(0).contiguous())[0]
    Ws = [pt2q.fill_synthetic((5120 if z % 3 else 13824, m), 900 + z, std=0.02).bfloat16() for z in range(count)]
    for _ in range(reps):
        outs = pt2q.engine.quantize_perchannel_group(Ws, [S1d] * count)
    torch.cuda.synchronize()
    print("pcg done", int(outs[0].iters[0]))
elif kind == "pc":
    n, m, count = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    X = pt2q.fill_synthetic((4096, m), 78, outliers=True).bfloat16()
    G = pt2q.gram(X)
    Ws = [pt2q.fill_synthetic((n, m), 900 + z, std=0.02).bfloat16() for z in range(count)]
    for _ in range(reps):
        outs = [pt2q.engine.quantize_blocks(W, G, None, block_size=m) for W in Ws]
    torch.cuda.synchronize()
    print("pc done", int(outs[0].iters[0]))
else:
    n, m, count = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    X = pt2q.fill_synthetic((4 * m, m), 78, outliers=True).half()
    G = pt2q.gram(X)
    Hinv, spd = pt2q.hessian_inverse(G, 4 * m)
    Ws = [pt2q.fill_synthetic((n, m), 900 + z, std=0.02).half() for z in range(count)]
    for _ in range(reps):
        outs = pt2q.engine.quantize_blocks_group(Ws, [G] * count, [Hinv] * count)
    torch.cuda.synchronize()
    print("group done", spd)

"""Dev probe: InfoNCE fwd/bwd and retrieval-rank kernel timing at cfg-5 scale on one GPU."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ceo-recommender_amd")]
import torch
from ceo_firm_matching.contrastive import _NCE, retrieval_ranks

dev = torch.device("cuda:0")
for B in [int(x) for x in (sys.argv[1:] or ["16384", "100000"])]:
    D = 256
    g = torch.Generator(device=dev).manual_seed(0)
    f = torch.nn.functional.normalize(torch.randn(B, D, device=dev, generator=g), dim=1)
    c = torch.nn.functional.normalize(torch.randn(B, D, device=dev, generator=g), dim=1)
    h = _NCE(f, c, B, B, D, 0, B, 0.07)
    def fwd():
        col = h.forward(h.norms())
        return h.loss(col)
    fwd(); h.backward(); torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    reps = 3
    e[0].record()
    for _ in range(reps): loss, st = fwd()
    e[1].record()
    for _ in range(reps): df, dc = h.backward()
    e[2].record()
    for _ in range(reps): r = retrieval_ranks(f, c, cap=None)
    e[3].record()
    torch.cuda.synchronize()
    tf, tb, tr = (e[i].elapsed_time(e[i + 1]) / reps for i in range(3))
    fl = 2.0 * B * B * D
    print(f"B={B} D={D}: fwd {tf:.2f} ms ({fl / tf / 1e9:.1f} TF/s)  bwd {tb:.2f} ms ({2 * fl / tb / 1e9:.1f} TF/s)  "
          f"ranks {tr:.2f} ms ({fl / tr / 1e9:.1f} TF/s)  loss={loss.item():.5f} status={st.item()}", flush=True)
    del h, df, dc
    torch.cuda.empty_cache()

"""Repeat bench.cosine_roofline in one process (run-to-run spread of the cosine leg)."""
import sys, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "ceo-recommender_amd")]
import torch, bench
dev = torch.device("cuda:0")
for i in range(6):
    r = bench.cosine_roofline(dev, D=128)
    print(i, r["avg_us"], r["achieved"], r["stream_peak_measured"], r["frac_of_measured_stream"], flush=True)

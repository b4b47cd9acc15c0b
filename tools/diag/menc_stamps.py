#!/usr/bin/env python3
"""Stage timing of the fused motion encoder from s_memrealtime marks (sa_raft_motion_encoder_stamps).

    python tools/diag/menc_stamps.py [--batch 1]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--variant", type=int, default=-1, help="sa_raft_motion_encoder_variant (1, 2; -1 default)")
    a = ap.parse_args()
    import torch
    from stereoalgorithms_amd import ops as O
    from stereoalgorithms_amd._native import dev
    torch.manual_seed(0)
    b, h, w = a.batch, 120, 160
    f1 = torch.randn(b, h, w, 256, device="cuda").half()
    f2 = torch.randn(b, h, w, 256, device="cuda").half()
    buf, _ = O.corr1d_pyramid(f1, f2, levels=4)
    flow = torch.randn(b, h, w, device="cuda") * 5
    ws = [torch.randn(64, 36, 1, 1), torch.randn(64), torch.randn(64, 2, 7, 7), torch.randn(64),
          torch.randn(64, 64, 3, 3), torch.randn(64), torch.randn(64, 64, 3, 3), torch.randn(64),
          torch.randn(126, 128, 3, 3), torch.randn(126)]
    ws = [x.cuda() * 0.05 for x in ws]
    blocks = b * (h // 8) * (w // 16)
    st = torch.zeros(blocks * 8 * 64, dtype=torch.int64, device="cuda")
    for rep in range(3):
        dev().sa_raft_motion_encoder_stamps(st.data_ptr() if rep == 2 else None)
        O.raft_motion_encoder(buf, flow, b, h, w, w, *ws, variant=a.variant)
        torch.cuda.synchronize()
    dev().sa_raft_motion_encoder_stamps(None)
    # kernel time without stamps (events around 20 back-to-back launches)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        O.raft_motion_encoder(buf, flow, b, h, w, w, *ws, variant=a.variant)
    e1.record()
    torch.cuda.synchronize()
    print(f"variant {a.variant}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per launch (incl. weight packing)")
    t = st.view(blocks, 8, 64)[:, :7, 0].double()
    d = (t[:, 1:] - t[:, :-1]) / 100.0  # s_memrealtime ticks at 100 MHz -> us
    names = ["flow patch", "lookup+flow taps", "stage-1 GEMM", "stage-2 convs", "stage-3 loop", "epilogue+store"]
    print(f"batch {b}, {blocks} workgroups: mean / max us per stage")
    for i, n in enumerate(names):
        print(f"  {n:18s} {d[:, i].mean().item():8.2f} {d[:, i].max().item():8.2f}")
    tot = (t[:, 6] - t[:, 0]) / 100.0
    span = (t[:, 6].max() - t[:, 0].min()) / 100.0
    print(f"  per-workgroup total {tot.mean().item():.2f} us (max {tot.max().item():.2f}); kernel span {span.item():.2f} us")


if __name__ == "__main__":
    main()

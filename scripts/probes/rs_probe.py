"""Row-scale GEMM probe: per-row error map of gemm4w RS 1 vs fp32 (debugging aid)."""
import sys
import torch
sys.path.insert(0, ".")
from llm_weighted_consensus_amd import ops

dev = torch.device("cuda:0")
for M, N, K, bn in [(300, 4096, 256, 256), (512, 4096, 256, 256), (300, 512, 256, 256), (256, 512, 64, 256),
                    (300, 1536, 256, 192)]:
    torch.manual_seed(0)
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    rs = torch.rand(M, device=dev) * 2 + 0.1
    ref = A.float() @ W.float().t()
    out = ops.gemm4w(A, W, bn=bn, rs=rs).float()
    torch.cuda.synchronize()
    ratio = (out / ref).median(dim=1).values  # ~ the scale the kernel applied per row
    bad = ((out - rs[:, None] * ref).abs() > 0.05 + 0.02 * (rs[:, None] * ref).abs()).any(1)
    idx = bad.nonzero().flatten().tolist()
    print(M, N, K, bn, "bad rows", len(idx), idx[:8], "...", idx[-4:], flush=True)
    for r in idx[:6]:
        print("   row", r, "applied", round(ratio[r].item(), 4), "want", round(rs[r].item(), 4),
              "rs of", [i for i in range(M) if abs(rs[i].item() - ratio[r].item()) < 1e-3][:3], flush=True)

import torch
for M, N, K in [(131584, 1024, 1024), (131584, 3072, 1024), (131584, 4096, 1024), (131584, 1024, 4096)]:
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    for _ in range(2):
        torch.matmul(x, w.t())
torch.cuda.synchronize()

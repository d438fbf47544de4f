import torch, time
n = 60000
K = torch.empty((n, n), dtype=torch.float64, device="cuda")
for _ in range(2): K.fill_(1.0)
torch.cuda.synchronize(); t0 = time.perf_counter()
for _ in range(3): K.fill_(0.5)
torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 3
print(f"fill 28.8 GB: {dt*1e3:.2f} ms = {K.numel()*8/dt/1e12:.2f} TB/s")

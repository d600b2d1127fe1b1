"""hipBLASLt int8 GEMM (torch._int_mm) throughput on one MI355X: the library's practical int8 MFMA
rate, to compare with the nominal 5033 TOP/s dense peak.  Measurement only."""
import torch

for n in (4096, 8192, 16384):
    a = torch.randint(-128, 128, (n, n), dtype=torch.int8, device="cuda")
    b = torch.randint(-128, 128, (n, n), dtype=torch.int8, device="cuda")
    for _ in range(3):
        torch._int_mm(a, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = max(3, int(2e13 // (2 * n ** 3)))
    e0.record()
    for _ in range(reps):
        torch._int_mm(a, b)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    tops = 2 * n ** 3 / (ms * 1e-3) / 1e12
    print(f"torch._int_mm {n}^3: {ms:.3f} ms  {tops:.1f} TOP/s  {tops / 5033.1648:.3f} of 5033", flush=True)

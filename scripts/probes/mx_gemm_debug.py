"""Debug: mi_op_gemm_mx with host-made e4m3 codes, (1) unit scales, (2) random scales."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd")]
import numpy as np, torch
from miclip import _native as N
from oracle import mx_ref
L = N.lib(); dev = torch.device("cuda:0"); sp = torch.cuda.current_stream().cuda_stream
rng = np.random.default_rng(0)
M, Nn, K = 256, 256, 256
qa = (rng.integers(0, 0x40, (M, K)) | (rng.integers(0, 2, (M, K)) << 7)).astype(np.uint8)
qw = (rng.integers(0, 0x40, (Nn, K)) | (rng.integers(0, 2, (Nn, K)) << 7)).astype(np.uint8)
for mode in ("unit", "rand"):
    sa = np.full((M, K // 64), 127, np.uint8) if mode == "unit" else rng.integers(124, 131, (M, K // 64)).astype(np.uint8)
    sw = np.full((Nn, K // 64), 127, np.uint8) if mode == "unit" else rng.integers(124, 131, (Nn, K // 64)).astype(np.uint8)
    t = [torch.from_numpy(x).to(dev) for x in (qa, mx_ref.to_stage_major(sa), qw, mx_ref.to_stage_major(sw))]
    out = torch.empty(M, Nn, device=dev)
    N.check(L.mi_op_gemm_mx(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), None, out.data_ptr(), M, Nn, K, 3, sp), "g")
    torch.cuda.synchronize()
    ref = mx_ref.gemm(qa, sa, qw, sw)
    got = out.cpu().numpy()
    err = np.abs(got - ref)
    print(mode, "max err", err.max(), "ref max", np.abs(ref).max())
    if err.max() > 1e-3 * np.abs(ref).max():
        bad = np.argwhere(err > 1e-3 * np.abs(ref).max())
        print(" bad count", len(bad), "first", bad[:8].tolist())
        print(" rows with errors", np.unique(bad[:, 0])[:40].tolist())
        print(" cols with errors", np.unique(bad[:, 1])[:40].tolist())
        # try hypotheses: transposed?
        print(" err vs ref.T", np.abs(got - ref.T).max())

# identity probe: A[m][k] = 1.0 if k == m % 128 (K = 128) -> out[m][n] = W[n][m % 128]
M, Nn, K = 256, 256, 128
qa = np.zeros((M, K), np.uint8)
qa[np.arange(M), np.arange(M) % K] = 0x38
wv = (np.arange(Nn * K).reshape(Nn, K) % 13).astype(np.float64)   # small ints, exact in e4m3
codes = {v: c for c, v in enumerate(mx_ref.E4M3) if not np.isnan(v)}
qw = np.vectorize(lambda v: codes[float(v)])(wv).astype(np.uint8)
sa = np.full((M, K // 64), 127, np.uint8); sw = np.full((Nn, K // 64), 127, np.uint8)
t = [torch.from_numpy(x).to(dev) for x in (qa, mx_ref.to_stage_major(sa), qw, mx_ref.to_stage_major(sw))]
out = torch.empty(M, Nn, device=dev)
N.check(L.mi_op_gemm_mx(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), None, out.data_ptr(), M, Nn, K, 3, sp), "g")
torch.cuda.synchronize()
got = out.cpu().numpy()
exp = wv[:, np.arange(M) % K].T
print("identity max err", np.abs(got - exp).max())
for m in range(0, 40, 1):
    row = got[m, :4]
    # which k of W does each output pick? find k with W[n][k] == got for n = 0..3 (ambiguous mod 13)
    cand = [int(k) for k in range(K) if np.allclose(wv[:4, k], row)]
    print(m, row.tolist(), "k candidates", cand[:6])

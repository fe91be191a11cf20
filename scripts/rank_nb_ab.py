"""rank_reg ring depth A/B: the product library's 8-slot ring against the A/B
build's 9-slot / 7-in-flight ring (MICLIP_RANK_NB=9), 1M x 512 f32, Q = 32,
k = 10, HIP events over 50 calls each, interleaved rounds."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd"), ROOT]
import torch  # noqa: E402
from miclip import _native as N, weights  # noqa: E402

Nr, D, Q, k = 1_000_000, 512, 32, 10
c = torch.from_numpy(weights.synthetic_corpus(Nr, D)).cuda()
q = torch.from_numpy(weights.synthetic_corpus(Q, D, seed=3)).cuda()


def run(L, reps):
    ws = torch.empty(L.mi_rank_workspace_bytes(Nr, Q, k), dtype=torch.uint8, device="cuda")
    s = torch.empty(Q, k, device="cuda")
    i = torch.empty(Q, k, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(reps + 3):
        if r == 3:
            e0.record()
        rc = L.mi_rank_topk(c.data_ptr(), Nr, D, 0, q.data_ptr(), Q, k, 0, 0, 0, s.data_ptr(), i.data_ptr(),
                            ws.data_ptr(), ws.numel(), st)
        assert rc == 0, L.mi_last_error()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3, s.clone(), i.clone()


prod, ab = N.lib(), N.lib_ab()
for rnd in range(3):
    os.environ.pop("MICLIP_RANK_NB", None)
    t8, s8, i8 = run(prod, 50)
    os.environ["MICLIP_RANK_NB"] = "9"
    t9, s9, i9 = run(ab, 50)
    print(f"round {rnd}: 8-slot (product) {t8:.1f} us, 9-slot (A/B) {t9:.1f} us, identical {torch.equal(s8, s9) and torch.equal(i8, i9)}")

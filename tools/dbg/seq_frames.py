import os, sys, numpy as np, torch
sys.path.insert(0, sys.argv[1] if len(sys.argv) > 1 else ".")
import oracle
from stereo_matching_amd import SGM, synthetic
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
H, W, D = 375, 1242, 128
PAIRS = [synthetic.stereo_pair(H, W, D, pair_index=i) for i in range(3)]
refs = [oracle.process(l, r, D)["lr"] for l, r in PAIRS]
st = torch.cuda.current_stream(dev)
def bits(t): return np.ascontiguousarray(t.cpu().numpy() if isinstance(t, torch.Tensor) else t).view(np.uint32)
sgm = SGM(H, W, 1, D, device=0)
for mode in ("fresh-empty", "fresh-nan", "sync"):
    for k, (l, r) in enumerate(PAIRS):
        dl, dr = torch.from_numpy(l).to(dev), torch.from_numpy(r).to(dev)
        out = torch.empty((H, W), dtype=torch.float32, device=dev)
        if mode == "fresh-nan":
            out.fill_(float("nan"))
        sgm.process_device(dl.data_ptr(), dr.data_ptr(), out.data_ptr(), stream=st.cuda_stream)
        torch.cuda.synchronize(dev)
        g = bits(out); w = bits(refs[k])
        bad = np.argwhere(g != w)
        print(mode, k, "mismatch", len(bad), bad[:5].tolist(), flush=True)
# host API
for k, (l, r) in enumerate(PAIRS):
    sgm.process(l, r)
    print("host", k, "mismatch", int((bits(sgm.get_lr_disp()) != bits(refs[k])).sum()), flush=True)
# fresh handle per pair
for k, (l, r) in enumerate(PAIRS):
    with SGM(H, W, 1, D, device=0) as s:
        s.process(l, r)
        print("fresh handle", k, "mismatch", int((bits(s.get_lr_disp()) != bits(refs[k])).sum()), flush=True)

"""Debug aid: device STOI envelopes vs the oracle's, per frame (GPU box)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from oracle import stoi_ref as S
from classical_speech_enhancement_amd import metrics
from classical_speech_enhancement_amd.synth import make_pair

sec = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
clean, noisy = make_pair(int(sec * 10), seconds=sec)
y = noisy.astype(np.float32).astype(np.float64)
x10 = S.resample_oct(clean, 10000, 16000)
y10 = S.resample_oct(y, 10000, 16000)
xs, ys = S.remove_silent_frames(x10, y10)
xt = S.band_envelopes(S.stft(xs)).T
yt = S.band_envelopes(S.stft(ys)).T
plan = metrics.StoiPlan(torch.as_tensor(clean).cuda().view(1, -1))
yd = torch.as_tensor(np.concatenate([y, clean]).astype(np.float32)).cuda()
v = plan.score(yd, [0, len(y)], [0, 0], clip=False)
M = xt.shape[0]
env = plan._scratch.view(torch.float64)[:2 * (len(x10) // 128 - 2) * 16].view(2, -1, 16)[:, :M, :15].cpu().numpy()
print("stoi dev", v, "oracle", S.stoi(clean, y, 16000), S.stoi(clean, clean, 16000))
for name, d, r in (("y", env[0], yt), ("x(cell path)", env[1], xt)):
    rel = np.abs(d - r).max(axis=1) / (np.abs(r).max(axis=1) + 1e-30)
    bad = np.nonzero(rel > 1e-4)[0]
    print(name, "M", M, "max rel per frame", rel.max(), "bad frames", bad[:40])
    if len(bad):
        f = bad[0]
        print(" frame", f, "dev", d[f][:6], "ref", r[f][:6])


def layout(n_sig, L):
    a = lambda x: (x + 255) & ~255
    n10 = (L * 5 + 7) // 8
    F = (n10 - 256) // 128 + 1 if n10 >= 256 else 0
    Mmax = F - 1 if F > 1 else 0
    Jmax = Mmax - 29 if Mmax >= 30 else 0
    NBLK = (Mmax + 15) // 16
    o = 0
    out = {}
    for name, size in (("coef64", 5 * 128 * 8), ("meta", n_sig * 16),
                       ("x10", n_sig * n10 * 8), ("en", n_sig * F * 8), ("kf", n_sig * F * 4),
                       ("btab", n_sig * NBLK * 72 * 4), ("xtob", n_sig * Mmax * 128),
                       ("xstat", n_sig * Jmax * 512)):
        out[name] = (o, size)
        o = a(o + size)
    return out, Mmax, Jmax


lay, Mmax, Jmax = layout(1, len(clean))
ws = plan.ws.cpu().numpy()
def arr(name, dt):
    o, s = lay[name]
    return ws[o:o + s].view(dt)
meta = arr("meta", np.int32)
print("meta", meta, "Mmax", Mmax, "Jmax", Jmax)
x10d = arr("x10", np.float64)
print("x10 max err", np.abs(x10d - x10).max())
kfd = arr("kf", np.int32)[:meta[0]]
w = S.hann_matlab(256)
e = np.array([20 * np.log10(np.linalg.norm(w * x10[i:i + 256]) + S.EPS) for i in range(0, len(x10) - 255, 128)])
print("kf equal", np.array_equal(kfd, np.nonzero((e.max() - 40 - e) < 0)[0]))
xtd = arr("xtob", np.float64).reshape(Mmax, 16)[:M, :15].astype(np.float64)
rel = np.abs(xtd - xt).max(axis=1) / (np.abs(xt).max(axis=1) + 1e-30)
print("xtob max rel", rel.max(), np.nonzero(rel > 1e-5)[0][:20])
xst = arr("xstat", np.float64).reshape(Jmax, 16, 4)
J = M - 29
seg = np.array([xt[j:j + 30] for j in range(J)])  # J,30,15
nx = np.linalg.norm(seg, axis=1)
mx = seg.mean(axis=1)
inv = 1 / (np.linalg.norm(seg - mx[:, None, :], axis=1) + S.EPS)
for k, ref_ in enumerate((nx, mx, inv)):
    d = xst[:J, :15, k].astype(np.float64)
    print("xstat", k, np.abs(d - ref_).max() / np.abs(ref_).max())
envy = env[0]
print("phaseB from device envs", S.stoi_from_envelopes(xtd.T, envy.T), "oracle", S.stoi_from_envelopes(xt.T, yt.T))

import sys, numpy as np
sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parent.parent))
from oracle import oracle as O
g = dict(np.load(str(__import__("pathlib").Path(__file__).resolve().parent.parent / "tests/golden/k5.npz")))
w, h = int(g["width"]), int(g["height"])
cam, sph, seeds = g["camera"], g["spheres"], g["seeds"]
rng = np.random.default_rng(1)
tiles = [(int(rng.integers(0, w // 8)), int(rng.integers(0, h // 8))) for _ in range(148)]
lens = []
for (tx, ty) in tiles:
    tl = []
    for k in range(64):
        x, y = tx * 8 + (k & 7), ty * 8 + (k >> 3)
        _, segs = O.render_pixels(np.zeros((1, 4), np.float32), np.array([x]), np.array([y]), cam, sph, seeds[:1])
        tl.append(segs)
    lens.append(tl)
L = np.array(lens)  # tiles x 64
print("mean path length", L.mean(), "hist", np.bincount(L.ravel(), minlength=9))
print("mean over tiles of max per tile", L.max(1).mean())
# wave-iterations without compaction: sum over bounce i of #waves with any lane alive at i
no_comp = sum((L > i).any(1).sum() for i in range(8)) / len(L)
# with compaction over groups of 4 tiles: sum over i of ceil(alive_i / 64)
G = L[:148].reshape(-1, 4 * 64)
comp = sum(np.ceil((G > i).sum(1) / 64).sum() for i in range(8)) / G.shape[0] / 4
print("wave-bounces per tile: without compaction", no_comp, "with 4-tile compaction", comp, "ideal", L.mean())
for i in range(8):
    print(i, "alive frac", round((L > i).mean(), 3), "waves busy no-comp", round((L > i).any(1).mean(), 3), "comp", round(np.ceil((G > i).sum(1) / 64).sum() / G.shape[0] / 4, 3))

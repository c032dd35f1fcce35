"""fit the scene the reference's three microfacet renders were made with
(img/microfacet*.png, README.md:301; no checkout scene reproduces them, tests/golden/ref_render_sweep.json),
then compare the Cook-Torrance sphere (interactions.cu:238-435) against them.

  refs  (here)     python tools/microfacet_fit.py refs
                   16x16-pixel tile means of the three images -> tests/golden/microfacet_ref_tiles.npz
  fit   (GPU box)  python tools/microfacet_fit.py fit --out gpurun_out/microfacet_fit.json
                   per image, coordinate descent over the scene parameters the renders differ in
                   (eye distance, field of view, light size / height / emittance, sphere size and position) on the tiles whose
                   pixels do not see the sphere (first hits from pt_test_camera + pt_test_intersect):
                   those tiles are diffuse + emissive light only, both already pinned to the reference
                   (tests/test_ref_renders.py).  200x200 at 256 spp while searching; the best point is
                   re-rendered at 800x800 and every tile compared, the sphere's tiles separately.
  table (here)     python tools/microfacet_fit.py table gpurun_out/microfacet_fit.json
                   -> tests/golden/microfacet_fit.json (the residual table)
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
IMAGES = {"microfacet_metallic_0.5_roughness_0.01.png": (0.5, 0.01),
          "microfacets_metallic_0.1_roughness_0.9.png": (0.1, 0.9),
          "microfacets_metallic_0.9_roughness_0.01.png": (0.9, 0.01)}
TILES = os.path.join(REPO, "tests", "golden", "microfacet_ref_tiles.npz")
NT = 50   # tiles per side
# parameter -> (start, first step, lower, upper)
PARAMS = {"eye_z": (10.5, 2.0, 4.0, 30.0), "light_s": (3.0, 1.0, 0.5, 9.5), "light_y": (10.0, 0.15, 9.0, 10.0),
          "sphere_s": (4.0, 0.8, 0.5, 8.0), "sphere_y": (4.0, 0.8, 0.5, 8.0), "sphere_x": (0.0, 0.8, -3.0, 3.0),
          "sphere_z": (0.0, 0.8, -3.0, 3.0), "fovy": (45.0, 5.0, 20.0, 70.0), "emit": (10.0, 4.0, 2.0, 60.0),
          "light_sz": (1.0, 0.25, 0.3, 3.0)}


def tiles_of(rgb, n=NT):
    h, w, _ = rgb.shape
    t = h // n
    return rgb.reshape(n, t, n, t, 3).astype(np.float64).mean(axis=(1, 3))


def refs(_):
    from PIL import Image
    out = {}
    for name in IMAGES:
        out[name] = tiles_of(np.asarray(Image.open(os.path.join("/root/reference/img", name)).convert("RGB"))).astype(np.float32)
    np.savez_compressed(TILES, **out)
    print("wrote", TILES)


def scene_json(p, metallic, roughness):
    with open(os.path.join(REPO, "scenes", "cornell_microfacet_test.json")) as f:
        d = json.load(f)
    d["Camera"]["EYE"] = [0.0, 5.0, p["eye_z"]]
    d["Camera"]["FOVY"] = p["fovy"]
    d["Materials"]["microfacet_mat"].update({"METALLIC": metallic, "ROUGHNESS": roughness})
    d["Materials"]["light"]["EMITTANCE"] = p["emit"]
    for o in d["Objects"]:
        if o["MATERIAL"] == "light":
            o["SCALE"] = [p["light_s"], 0.3, p["light_s"] * p["light_sz"]]
            o["TRANS"] = [0.0, p["light_y"], 0.0]
        if o["MATERIAL"] == "microfacet_mat":
            o["SCALE"] = [p["sphere_s"]] * 3
            o["TRANS"] = [p["sphere_x"], p["sphere_y"], p["sphere_z"]]
    return d


class Renderer:
    def __init__(self):
        sys.path.insert(0, os.path.join(REPO, "project3-cuda-path-tracer-2025_amd"))
        import ptamd
        self.P = ptamd
        self.tmp = tempfile.mkdtemp()

    def render(self, d, res, spp, sphere_mask=True):
        from PIL import Image
        P = self.P
        path = os.path.join(self.tmp, "s.json")
        with open(path, "w") as f:
            json.dump(d, f)
        sc = P.SceneFile(path, res=(res, res))
        tr = P.PathTracer(sc)
        mask = None
        if sphere_mask:   # tiles with a pixel whose first hit is the sphere (material id of microfacet_mat)
            cam = tr.test_camera(1)
            hits = tr.test_intersect(cam)
            mid = sc.material_names.index("microfacet_mat")
            sph = (hits["t"] > 0) & (hits["materialId"] == mid)
            sph = sph.reshape(res, res)[:, ::-1]          # saveImage mirrors x
            t = res // NT
            mask = sph.reshape(NT, t, NT, t).any(axis=(1, 3))
        tr.trace_frames(1, spp)
        P.save_png(tr.image(), res, res, spp, os.path.join(self.tmp, "x"))
        rgb = np.asarray(Image.open(os.path.join(self.tmp, "x.png")).convert("RGB"))
        tr.free()
        sc.close()
        return tiles_of(rgb), mask


def dist(ours, ref, mask):
    d = np.abs(ours - ref).mean(axis=2)
    keep = ~mask
    # one tile ring around the sphere is left out too (its edge pixels, the contact shadow)
    grown = mask.copy()
    grown[1:] |= mask[:-1]; grown[:-1] |= mask[1:]; grown[:, 1:] |= mask[:, :-1]; grown[:, :-1] |= mask[:, 1:]
    keep = ~grown
    return float(d[keep].mean()), keep


def fit(args):
    ref_tiles = np.load(TILES)
    R = Renderer()
    report = {}
    for name, (met, rough) in IMAGES.items():
        ref = ref_tiles[name].astype(np.float64)
        p = {k: v[0] for k, v in PARAMS.items()}
        step = {k: v[1] for k, v in PARAMS.items()}
        cache = {}

        def score(q):
            key = tuple(round(q[k], 4) for k in PARAMS)
            if key not in cache:
                ours, mask = R.render(scene_json(q, met, rough), args.res, args.spp)
                cache[key] = dist(ours, ref, mask)[0]
            return cache[key]

        best = score(p)
        for rnd in range(args.rounds):
            improved = False
            for k in PARAMS:
                for sgn in (1, -1):
                    q = dict(p)
                    q[k] = min(PARAMS[k][3], max(PARAMS[k][2], p[k] + sgn * step[k]))
                    s = score(q)
                    if s < best - 1e-3:
                        best, p, improved = s, q, True
                        break
            if not improved:
                step = {k: v * 0.5 for k, v in step.items()}
            print(f"{name} round {rnd}: {best:.3f} {json.dumps({k: round(v, 3) for k, v in p.items()})}", flush=True)
        ours, mask = R.render(scene_json(p, met, rough), 800, args.final_spp)
        d = np.abs(ours - ref)
        wall, keep = dist(ours, ref, mask)
        sph = d[mask]
        report[name] = {"metallic": met, "roughness": rough, "params": {k: round(v, 4) for k, v in p.items()},
                        "search": {"res": args.res, "spp": args.spp, "evaluations": len(cache), "best_wall_mean_abs": round(best, 3)},
                        "final": {"res": 800, "spp": args.final_spp,
                                  "wall_tiles": int(keep.sum()), "wall_mean_abs": round(wall, 3),
                                  "wall_max_abs": round(float(d.mean(axis=2)[keep].max()), 3),
                                  "sphere_tiles": int(mask.sum()),
                                  "sphere_mean_abs": round(float(sph.mean()), 3) if sph.size else None,
                                  "sphere_max_abs": round(float(sph.mean(axis=1).max()), 3) if sph.size else None,
                                  "sphere_signed_mean": [round(float(x), 3) for x in (ours - ref)[mask].mean(axis=0)] if sph.size else None,
                                  "all_mean_abs": round(float(d.mean()), 3)}}
        print(json.dumps({name: report[name]["final"]}), flush=True)
    with open(args.out, "w") as f:
        json.dump(report, f, indent=1)


def table(args):
    with open(args.fit) as f:
        rep = json.load(f)
    out = {"source": "tools/microfacet_fit.py fit (GPU) on tests/golden/microfacet_ref_tiles.npz",
           "bars": "tests/test_ref_renders.py: whole image mean |tile diff| < 0.4 of 255, specular tiles mean < 0.6, "
                   "max < 2, |signed mean| < 0.35",
           "images": rep}
    dst = os.path.join(REPO, "tests", "golden", "microfacet_fit.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    for n, r in rep.items():
        print(n, r["params"], r["final"])


def main():
    ap = argparse.ArgumentParser()
    sp = ap.add_subparsers(dest="cmd", required=True)
    sp.add_parser("refs")
    p = sp.add_parser("fit")
    p.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "microfacet_fit.json"))
    p.add_argument("--res", type=int, default=200)
    p.add_argument("--spp", type=int, default=256)
    p.add_argument("--rounds", type=int, default=24)
    p.add_argument("--final-spp", type=int, default=2000)
    p = sp.add_parser("table")
    p.add_argument("fit")
    a = ap.parse_args()
    {"refs": refs, "fit": fit, "table": table}[a.cmd](a)


if __name__ == "__main__":
    main()

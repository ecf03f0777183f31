"""CPU micro-benchmark of LeRobotWriter's host work (experiment tooling): synthetic episodes with
every feature of the default set (PNG bytes are random blobs of the measured mean size), written
unthreaded to a temp dir; prints the writer's timing split and the meta/stats.json digest so two
versions of the writer can be compared for speed and identical output."""
import argparse
import hashlib
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mujoco_manip_amd import dataset as D  # noqa: E402


def make_episodes(n, image_size, seed=0, png_frames=False):
    rng = np.random.default_rng(seed)
    feats = D._features_at(D.resolve_features(None), image_size)
    eps = []
    for e in range(n):
        L = int(rng.integers(70, 110))
        obj, bn = D.TASK_SETS["all"][e % 9]
        ep = D.Episode(e, obj, bn, None)
        ep.length = L
        for k, f in feats.items():
            if k in D.IMAGE_KEYS:
                files = [rng.bytes(int(rng.integers(5000, 8000))) for _ in range(L)]
                if png_frames:  # as collect_episodes hands them over (one buffer per episode)
                    offs = np.zeros(L + 1, np.int64)
                    np.cumsum([len(b) for b in files], out=offs[1:])
                    files = D.PngFrames(np.frombuffer(b"".join(files), np.uint8).copy(), offs)
                ep.frames[k] = files
                fs = np.zeros((L, 4, 3))
                fs[:, 0] = rng.integers(0, 40, (L, 3)) / 255.0
                fs[:, 1] = rng.integers(200, 256, (L, 3)) / 255.0
                fs[:, 2] = rng.integers(10**6, 10**7, (L, 3)) / 255.0
                fs[:, 3] = rng.integers(10**8, 10**9, (L, 3)) / (255.0 * 255.0)
                ep.image_stats[k] = D._merge_image_stats(fs, image_size * image_size)
            elif f["dtype"] == "string":
                ep.frames[k] = [D.phase_description(int(s), obj, bn) for s in rng.integers(0, 10, L)]
            else:
                ep.frames[k] = rng.standard_normal((L,) + tuple(f["shape"])).astype(np.float32)
        eps.append(ep)
    return feats, eps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, default=1024)
    ap.add_argument("--image-size", type=int, default=128)
    ap.add_argument("--list-frames", action="store_true", help="PNG files as lists of bytes (default: PngFrames)")
    a = ap.parse_args()
    feats, eps = make_episodes(a.episodes, a.image_size, png_frames=not a.list_frames)
    with tempfile.TemporaryDirectory() as root:
        w = D.LeRobotWriter(os.path.join(root, "ds"), "u/bench", feats, threaded=False, io_threads=0)
        t0 = time.perf_counter()
        for ep in eps:
            w.add_episode(ep)
        w.close()
        dt = time.perf_counter() - t0
        stats = open(os.path.join(root, "ds", "meta", "stats.json"), "rb").read()
        import pyarrow.parquet as pq
        ep_meta = pq.read_table(os.path.join(root, "ds", "meta", "episodes", "chunk-000", "file-000.parquet"))
        meta_digest = hashlib.sha256(json.dumps(ep_meta.to_pylist(), sort_keys=True, default=str).encode()).hexdigest()
    print(json.dumps({"episodes": a.episodes, "seconds": round(dt, 3), "ms_per_episode": round(1e3 * dt / a.episodes, 3),
                      "timing": {k: round(v, 3) for k, v in w.timing.items()},
                      "stats_sha256": hashlib.sha256(stats).hexdigest()[:16], "episodes_meta_sha256": meta_digest[:16]}))


if __name__ == "__main__":
    main()

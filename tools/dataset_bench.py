"""f2 throughput probe: generate a LeRobot dataset with camera images from batched expert episodes
and report frames/s, PNG bytes, peak host RSS and device memory over the run.

  python tools/dataset_bench.py --num-envs 8192 --episodes 8192 --image-size 128 --out gpurun_out/ds.json

Diagnostic tool; writes the dataset under --root (deleted afterwards unless --keep).
"""
import argparse
import json
import os
import resource
import shutil
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-envs", type=int, default=8192)
    ap.add_argument("--episodes", type=int, default=8192)
    ap.add_argument("--image-size", type=int, default=128)
    ap.add_argument("--root", default="/tmp/mmx_ds")
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "dataset_bench.json"))
    ap.add_argument("--keep", action="store_true")
    ap.add_argument("--image-compression", default="SNAPPY", choices=("SNAPPY", "NONE"))
    ap.add_argument("--io-threads", type=int, default=None, help="LeRobotWriter I/O lanes (default 4)")
    ap.add_argument("--no-write", action="store_true", help="collect only: the sink drops the episodes")
    ap.add_argument("--cprofile", default=None, help="cProfile the collecting thread into this .txt")
    a = ap.parse_args()

    import torch

    from mujoco_manip_amd import dataset as D

    free0, total = torch.cuda.mem_get_info()
    used = []

    def sample_memory():  # (no per-step hook: collect_episodes' on_step costs a host sync per step)
        f, _ = torch.cuda.mem_get_info()
        used.append(total - f)

    feats = D.resolve_features(None, "staged")
    shutil.rmtree(a.root, ignore_errors=True)
    path = os.path.join(a.root, "u", "bench")
    feats = D._features_at(feats, a.image_size)
    writer = D.LeRobotWriter(path, "u/bench", feats, threaded=True, image_compression=a.image_compression,
                             io_threads=a.io_threads)
    frames = [0]
    png_bytes = [0]

    def sink(ep):
        if ep.index % 64 == 0:
            sample_memory()
        frames[0] += ep.length
        if ep.index % 16 == 0:  # PNG size from every 16th episode (PngFrames: its buffer's size)
            png_bytes[0] += 16 * sum(D._png_nbytes(ep.frames.get(k, [])) for k in D.IMAGE_KEYS)
        if a.no_write:
            return
        writer.add_episode(ep)

    prof = None
    if a.cprofile:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    D.collect_episodes(a.episodes, D.TASK_SETS["all"], set(feats), randomize_objects=True, seed=0,
                       num_envs=a.num_envs, sink=sink, image_size=a.image_size)
    info = writer.close()
    dt = time.perf_counter() - t0
    if prof is not None:
        import io
        import pstats
        prof.disable()
        buf = io.StringIO()
        pstats.Stats(prof, stream=buf).sort_stats("tottime").print_stats(40)
        pstats.Stats(prof, stream=buf).sort_stats("cumulative").print_stats(40)
        open(a.cprofile, "w").write(buf.getvalue())
    if a.no_write:
        info = {"total_episodes": a.episodes, "total_frames": frames[0]}
    rss = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0  # MB (Linux: KB)
    size = sum(os.path.getsize(os.path.join(d, f)) for d, _, fs in os.walk(path) for f in fs)
    rec = {"config": {"num_envs": a.num_envs, "episodes": a.episodes, "image_size": a.image_size,
                      "png": "device (mmx_png_encode)", "image_compression": a.image_compression,
                      "writer": "none (--no-write)" if a.no_write else f"LeRobotWriter(threaded=True, io_threads={writer.io_threads})", "root": a.root, "features": "all (2 cameras, numeric, actions, reward, phase)"},
           "episodes": info["total_episodes"], "frames": info["total_frames"], "seconds": dt,
           "frames_per_s": info["total_frames"] / dt, "images_per_s": 2 * info["total_frames"] / dt,
           "png_mean_bytes": png_bytes[0] / max(2 * frames[0], 1), "dataset_bytes": size,
           "peak_host_rss_mb": rss, "device_used_mb_start": (total - free0) / 2**20,
           "device_used_mb_max": max(used) / 2**20 if used else None,
           "device_used_mb_min_after_start": min(used) / 2**20 if used else None,
           "host_cpus": len(os.sched_getaffinity(0)),
           "writer_timing": None if a.no_write else {k: round(v, 3) for k, v in writer.timing.items()}}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(rec, open(a.out, "w"), indent=1)
    print(json.dumps(rec))
    if not a.keep:
        shutil.rmtree(a.root, ignore_errors=True)


if __name__ == "__main__":
    main()

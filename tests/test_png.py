"""The batched HIP PNG encoder (mujoco_manip_amd/csrc/mmx_png.hip) used by the dataset writer.

Every file must be a valid PNG that any decoder reads back to exactly the input pixels: PIL
decodes it (PIL verifies each chunk's CRC-32), zlib inflates the IDAT stream (verifying the
Adler-32) to the filter-0 scanlines, and the chunk layout is walked by hand.  Inputs: random
(incompressible) images, flat and striped ones (long matches at both distances), rendered camera
images, and sizes that are not multiples of 16 or not square."""
import io
import struct
import zlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sim():
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    from mujoco_manip_amd import _lib

    s = _lib.Sim(1, action_mode="abs_pos", image_size=0)
    yield s
    s.close()


def _chunks(png: bytes):
    assert png[:8] == b"\x89PNG\r\n\x1a\n"
    k, out = 8, []
    while k < len(png):
        n = struct.unpack(">I", png[k:k + 4])[0]
        typ, data = png[k + 4:k + 8], png[k + 8:k + 8 + n]
        crc = struct.unpack(">I", png[k + 8 + n:k + 12 + n])[0]
        assert zlib.crc32(typ + data) & 0xFFFFFFFF == crc, typ
        out.append((typ, data))
        k += 12 + n
    assert k == len(png)
    return out


def _check(sim, imgs: np.ndarray):
    from PIL import Image

    packed, offs = sim.png_encode(torch.as_tensor(imgs).cuda())
    data = packed.cpu().numpy().tobytes()
    sizes = []
    for i, im in enumerate(imgs):
        png = data[offs[i]:offs[i + 1]]
        ch = _chunks(png)
        assert ch[0][0] == b"IHDR" and ch[-1][0] == b"IEND"
        w, h = struct.unpack(">II", ch[0][1][:8])
        assert (h, w) == im.shape[:2] and ch[0][1][8:] == b"\x08\x02\x00\x00\x00"
        raw = zlib.decompress(b"".join(d for t, d in ch if t == b"IDAT"))
        lines = np.frombuffer(raw, np.uint8).reshape(h, 3 * w + 1)
        assert (lines[:, 0] == 0).all()
        np.testing.assert_array_equal(lines[:, 1:].reshape(im.shape), im)
        np.testing.assert_array_equal(np.asarray(Image.open(io.BytesIO(png)).convert("RGB")), im)
        sizes.append(len(png))
    return np.array(sizes)


def test_png_random_and_structured(sim):
    rng = np.random.default_rng(0)
    S = 64
    noise = rng.integers(0, 256, (3, S, S, 3), dtype=np.uint8)
    flat = np.zeros((2, S, S, 3), np.uint8)
    flat[0] = (200, 30, 40)
    stripes = np.zeros((2, S, S, 3), np.uint8)
    stripes[0, :, ::2] = 255           # columns: the 3-byte distance breaks, the row above matches
    stripes[1, ::3] = (10, 250, 7)     # rows: the row above breaks, the 3-byte distance matches
    sz = _check(sim, np.concatenate([noise, flat, stripes]))
    raw = S * (3 * S + 1)
    assert sz[:3].max() < 1.13 * raw + 200  # incompressible: <= 9 bits per byte + framing
    assert sz[3:5].max() < 0.02 * raw + 200  # flat: whole rows as matches


@pytest.mark.parametrize("hw", [(84, 84), (100, 100), (224, 224), (37, 91), (1, 1), (1, 300)])
def test_png_sizes(sim, hw):
    h, w = hw
    rng = np.random.default_rng(h * 1000 + w)
    base = rng.integers(0, 256, (2, h, w, 3), dtype=np.uint8)
    base[1, h // 2:] = base[1, : h - h // 2]  # repeated rows
    _check(sim, base)


def test_png_rendered_frames_compress(sim):
    """Camera images of a C5-like batch (128 x 128) round-trip and compress well (flat shading)."""
    from mujoco_manip_amd import _lib
    from mujoco_manip_amd.vec_env import PickPlaceVecEnv

    env = PickPlaceVecEnv(8, tasks="all", action_mode="abs_pos", reward_type="staged", randomize_objects=True,
                          image_size=128)
    env.reset(seed=[_lib.episode_seed(5, i) for i in range(8)])
    for _ in range(20):
        obs, *_ = env.step(env.expert_plan(16))
    imgs = torch.cat([obs["image_overhead"], obs["image_wrist"]]).cpu().numpy()
    sz = _check(sim, imgs)
    ratio = (128 * 385) / sz.mean()
    print(f"mean PNG {sz.mean():.0f} B, compression {ratio:.1f}x")
    assert ratio > 3.0
    env.close()


def test_png_width_limit(sim):
    """The row-above match's deflate distance 3 W + 1 must stay <= 32768: the widest accepted
    image (W = 10922) round-trips, one pixel wider is rejected up front."""
    from mujoco_manip_amd import _lib

    rng = np.random.default_rng(7)
    im = rng.integers(0, 256, (1, 3, _lib.PNG_MAX_WIDTH, 3), dtype=np.uint8)
    im[0, 1] = im[0, 0]  # a whole row repeated: the match at the maximum distance
    _check(sim, im)
    assert sim.L.mmx_png_bound(_lib.PNG_MAX_WIDTH + 1, 2) == -1
    with pytest.raises(ValueError, match="unsupported image size"):
        sim.png_encode(torch.zeros((1, 2, _lib.PNG_MAX_WIDTH + 1, 3), dtype=torch.uint8, device="cuda"))


def test_png_encode_from_another_stream(sim):
    """png_encode called under another current stream: the encoder runs on the sim's
    stream, its inputs produced on the caller's stream are waited for, and the caller's stream sees
    the finished files; the bytes equal an encode on the default stream."""
    rng = np.random.default_rng(8)
    host = rng.integers(0, 256, (6, 48, 64, 3), dtype=np.uint8)
    want, woffs = sim.png_encode(torch.as_tensor(host).cuda())
    want = want.cpu().numpy()
    other = torch.cuda.Stream()
    with torch.cuda.stream(other):
        big = torch.randn(4096, 4096, device="cuda")
        for _ in range(4):  # keep the caller's stream busy before the images exist
            big = big @ big * 1e-3
        imgs = torch.as_tensor(host).cuda(non_blocking=True) + (big[0, 0] * 0).to(torch.uint8)
        packed, offs = sim.png_encode(imgs)
        got = packed.cpu().numpy()  # ordered on the caller's stream
    np.testing.assert_array_equal(offs, woffs)
    np.testing.assert_array_equal(got, want)


def test_png_encode_device_matches_host_path(sim):
    """png_encode_device (the dataset loop's sync-free form: files packed on the device, the end
    offsets left on the device, room for n bounds) gives the same files as png_encode, also for a
    strided batch (one camera of [n, 2, H, W, 3] images)."""
    rng = np.random.default_rng(9)
    host = rng.integers(0, 256, (5, 2, 40, 56, 3), dtype=np.uint8)
    host[:, :, 20:] = host[:, :, :20]  # repeated rows: matches at the row-above distance
    dev = torch.as_tensor(host).cuda()
    for cam in range(2):
        want, woffs = sim.png_encode(dev[:, cam].contiguous())
        packed, ends = sim.png_encode_device(dev[:, cam])
        ends = ends.cpu().numpy()
        assert packed.numel() == 5 * sim.L.mmx_png_bound(56, 40)
        np.testing.assert_array_equal(np.concatenate([[0], ends]), woffs)
        np.testing.assert_array_equal(packed[:int(ends[-1])].cpu().numpy(), want.cpu().numpy())


def test_image_stats_kernel_equals_torch_definition(sim):
    """mmx_image_stats (one HIP pass, dword-gathered channel bytes + v_dot4) equals the torch
    definition of the dataset's per-frame statistics bit for bit: aligned 4-pixel groups (128^2,
    224^2), sizes whose pixel count is not a multiple of 4 (byte path), a camera batch with a stride
    between images (the dataset's [N, 2, S, S, 3] images, one camera) and extreme values."""
    from mujoco_manip_amd import dataset as D

    rng = np.random.default_rng(21)
    cases = [rng.integers(0, 256, (7, 128, 128, 3), dtype=np.uint8),
             rng.integers(0, 256, (3, 224, 224, 3), dtype=np.uint8),
             rng.integers(0, 256, (4, 17, 23, 3), dtype=np.uint8),
             np.zeros((2, 16, 16, 3), np.uint8), np.full((2, 16, 16, 3), 255, np.uint8)]
    for imgs in cases:
        t = torch.as_tensor(imgs).cuda()
        got = sim.image_stats(t).cpu().numpy()
        x = imgs.reshape(len(imgs), -1, 3).astype(np.int64)
        want = np.stack([x.min(1), x.max(1), x.sum(1), (x * x).sum(1)], 1)
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(D._frame_image_stats_device(sim, t).cpu().numpy(),
                                      D._frame_image_stats(t).cpu().numpy())
    both = torch.as_tensor(rng.integers(0, 256, (5, 2, 64, 64, 3), dtype=np.uint8)).cuda()
    for cam in (0, 1):
        v = both[:, cam]
        assert v.stride(0) == 2 * 64 * 64 * 3
        np.testing.assert_array_equal(sim.image_stats(v).cpu().numpy(),
                                      sim.image_stats(v.contiguous()).cpu().numpy())

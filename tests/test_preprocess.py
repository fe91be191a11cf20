"""Frame preprocessing.

CPU: the oracle's restatement of Pillow's ImagingResample is bit-exact against
PIL itself (the reference's actual dependency: torchvision's Resize calls
PIL.Image.resize), the host Transform equals the oracle, and the library's
host coefficient routine equals the oracle's.  GPU: mi_preprocess_frames on
decoded uint8 frames equals the host Transform (PIL) bit for bit."""
import ctypes

import numpy as np
import pytest

from oracle import preprocess_ref as P

SIZES = [(720, 1280), (1280, 720), (375, 500), (224, 224), (80, 100), (224, 300), (33, 47)]


def _img(h, w, seed):
    rng = np.random.default_rng(seed)
    # random noise plus smooth structure (exercises clipping of the bicubic lobes)
    yy, xx = np.mgrid[0:h, 0:w]
    base = (127 + 120 * np.sin(xx / 7.0 + yy / 11.0))[..., None] * np.array([1.0, 0.7, 0.4])
    return np.clip(base + rng.normal(0, 40, (h, w, 3)), 0, 255).astype(np.uint8)


@pytest.mark.parametrize("hw", [(72, 128), (120, 50), (37, 41), (224, 224)])
def test_resample_oracle_matches_pil(hw):
    from PIL import Image
    img = _img(*hw, 0)
    for size in [(64, 36), (224, 224), (50, 90), (hw[1], 30), (300, hw[0])]:
        for f, pf in [(P.BICUBIC, Image.BICUBIC), (P.BILINEAR, Image.BILINEAR)]:
            ref = np.asarray(Image.fromarray(img).resize(size, pf))
            assert np.array_equal(P.resize(img, size, f), ref), (hw, size, f)


@pytest.mark.parametrize("hw", [(720, 1280), (375, 500), (224, 300)])
def test_host_transform_equals_oracle(hw):
    from PIL import Image
    from miclip.preprocess import Transform
    img = _img(*hw, 1)
    got = Transform(224)(Image.fromarray(img)).numpy()
    assert np.array_equal(got, P.clip_transform(img, 224))
    got = Transform(224, squash=True)(Image.fromarray(img)).numpy()
    assert np.array_equal(got, P.squash_transform(img, 224))


def test_resample_coeffs_abi_matches_oracle():
    from miclip import _native
    L = _native.lib()
    for in_size, out_size in [(1280, 398), (720, 224), (500, 298), (100, 224), (47, 47), (300, 224)]:
        for f in (P.BICUBIC, P.BILINEAR):
            kk = np.zeros(out_size * 64, np.int32)
            bd = np.zeros(out_size * 2, np.int32)
            ks = L.mi_resample_coeffs(in_size, 0.0, float(in_size), out_size, f, kk.ctypes.data, kk.size,
                                      bd.ctypes.data)
            rk, rb = P.coeffs(in_size, out_size, f)
            assert ks == rk.shape[1]
            assert np.array_equal(kk[:out_size * ks].reshape(out_size, ks), rk)
            assert np.array_equal(bd.reshape(out_size, 2), rb)
    assert L.mi_resample_coeffs(0, 0.0, 1.0, 4, 0, None, 0, None) < 0


@pytest.mark.gpu
@pytest.mark.parametrize("hw", SIZES)
@pytest.mark.parametrize("squash", [False, True])
def test_preprocess_frames_equals_pil(gpu, hw, squash):
    import torch
    from PIL import Image
    from miclip.preprocess import Transform, preprocess_frames
    B = 3
    imgs = [_img(*hw, 10 + i) for i in range(B)]
    frames = torch.from_numpy(np.stack(imgs)).to(gpu)
    got = preprocess_frames(frames, 224, squash=squash).cpu().numpy()
    tf = Transform(224, squash=squash)
    for i in range(B):
        ref = tf(Image.fromarray(imgs[i])).numpy()
        assert np.array_equal(got[i], ref), (hw, squash, i, np.abs(got[i] - ref).max())
    b16 = preprocess_frames(frames, 224, squash=squash, out_dtype=torch.bfloat16)
    assert torch.equal(b16.cpu(), torch.from_numpy(got).bfloat16())


@pytest.mark.gpu
def test_preprocess_batch_api_and_errors(gpu):
    import torch
    from PIL import Image
    from miclip import _native
    from miclip.preprocess import Transform, preprocess_frames
    imgs = [Image.fromarray(_img(360, 640, 20 + i)) for i in range(5)]
    tf = Transform(224)
    got = tf.batch(imgs, device=gpu).cpu().numpy()
    for i, im in enumerate(imgs):
        assert np.array_equal(got[i], tf(im).numpy())
    assert preprocess_frames(torch.zeros(0, 8, 8, 3, dtype=torch.uint8, device=gpu)).shape == (0, 3, 224, 224)
    with pytest.raises(_native.MiClipError):
        preprocess_frames(torch.zeros(1, 8, 8, 3, device=gpu))

"""Fresh-batch kernel (data_aug.hip) on MI355X against PyTorch: gather + normalise exactly,
crops / flips drawn from the torchvision RandomCrop(pad)+RandomHorizontalFlip set."""
import pytest
import torch

from garfield_amd.data.fresh import DeviceBatches

pytestmark = pytest.mark.gpu


def _normalised(src, mean, std):
    x = src.permute(0, 3, 1, 2).double() / 255.0
    return (x - torch.tensor(mean, dtype=torch.float64).view(1, -1, 1, 1)) / \
        torch.tensor(std, dtype=torch.float64).view(1, -1, 1, 1)


def test_gather_normalise_no_augmentation(cuda, native):
    g = torch.Generator().manual_seed(0)
    src = torch.randint(0, 256, (50, 8, 8, 3), dtype=torch.uint8, generator=g).to(cuda)
    idx = torch.randint(0, 50, (40,), generator=g).to(cuda)
    mean, std = [0.4, 0.5, 0.6], [0.2, 0.25, 0.3]
    out = torch.empty((40, 3, 8, 8), dtype=torch.bfloat16, device=cuda, memory_format=torch.channels_last)
    native.gpu_augment_gather(src, idx, 7, 0, mean, std, out, 0, False)
    ref = _normalised(src[idx].cpu(), mean, std)
    assert torch.allclose(out.double().cpu(), ref, atol=1e-2, rtol=1e-2)


def test_crop_flip_from_reference_candidate_set(cuda, native):
    g = torch.Generator().manual_seed(1)
    H = W = 8
    pad = 2
    src = torch.randint(0, 256, (20, H, W, 3), dtype=torch.uint8, generator=g).to(cuda)
    idx = torch.arange(20, device=cuda)
    mean, std = [0.5, 0.5, 0.5], [0.25, 0.25, 0.25]
    out = torch.empty((20, 3, H, W), dtype=torch.bfloat16, device=cuda, memory_format=torch.channels_last)
    native.gpu_augment_gather(src, idx, 3, 5, mean, std, out, pad, True)
    raw = src.permute(0, 3, 1, 2).double().cpu() / 255.0
    padded = torch.nn.functional.pad(raw, (pad, pad, pad, pad))             # black padding, then normalise
    o = out.double().cpu()
    crops_seen, flips_seen = set(), 0
    for r in range(20):
        best = None
        for oy in range(2 * pad + 1):
            for ox in range(2 * pad + 1):
                c = padded[r, :, oy:oy + H, ox:ox + W]
                for fl in (False, True):
                    cand = (((c.flip(2) if fl else c) - 0.5) / 0.25)
                    err = (cand - o[r]).abs().max().item()
                    if best is None or err < best[0]:
                        best = (err, oy, ox, fl)
        assert best[0] < 2e-2, (r, best)
        crops_seen.add((best[1], best[2]))
        flips_seen += best[3]
    assert len(crops_seen) > 3 and 0 < flips_seen < 20          # the offsets and flips actually vary
    out2 = torch.empty_like(out)
    native.gpu_augment_gather(src, idx, 3, 5, mean, std, out2, pad, True)
    assert torch.equal(out, out2)                                # (seed, step) reproduces the batch
    native.gpu_augment_gather(src, idx, 3, 6, mean, std, out2, pad, True)
    assert not torch.equal(out, out2)


def test_device_batches_feed_new_versions(cuda):
    feed = DeviceBatches.synthetic(1000, (3, 32, 32), 10, 4, 16, cuda, seed=2)
    b1 = feed.next()
    v1, x1 = b1[0][0]._version, b1[0][0].clone()
    b2 = feed.next()
    assert b2[0][0]._version != v1 and not torch.equal(b2[0][0], x1)
    assert len(b2) == 4 and b2[0][0].shape == (16, 3, 32, 32) and b2[0][1].shape == (16,)
    assert b2[0][0].is_contiguous(memory_format=torch.channels_last)


def test_hashed_sampling_labels_and_engine_buffers(cuda, native):
    """idx=None: the kernel draws the images itself and writes their labels; attach() makes the
    feed write straight into a consumer's buffers."""
    feed = DeviceBatches.synthetic(64, (3, 8, 8), 10, 2, 8, cuda, seed=4)
    x = torch.empty((16, 3, 8, 8), dtype=torch.bfloat16, device=cuda, memory_format=torch.channels_last)
    y = torch.empty(16, dtype=torch.long, device=cuda)
    assert feed.attach((x, y))
    b = feed.next()
    assert b[0][0].data_ptr() == x.data_ptr() and b[1][1].data_ptr() == y[8:].data_ptr()
    # every row is some image of the dataset (pad 0 / no flip reproduces it exactly) with its label
    feed2 = DeviceBatches(feed.src.cpu(), feed.labels.cpu(), 2, 8, cuda, pad=0, flip=False, seed=4)
    xs, ys = zip(*feed2.next())
    xs, ys = torch.cat(xs).double().cpu(), torch.cat(ys).cpu()
    ref = _normalised(feed.src.cpu(), feed2.mean, feed2.std)
    for r in range(16):
        err = (ref - xs[r]).abs().flatten(1).max(1).values
        j = int(err.argmin())
        assert err[j] < 2e-2 and int(feed.labels[j]) == int(ys[r])

"""FineWeb shard loader (gvl.data) vs the restated DataLoaderLite windows (oracle/data.py,
train_gpt2.py:148-187): rank-strided windows, shard rollover and wrap-around, reset; and
get_most_likely_row (train_gpt2.py:190-202) vs explicit per-ending arithmetic."""
import numpy as np
import pytest
import torch

from gvl.data import DataLoaderLite, get_most_likely_row
from oracle import data as OD


@pytest.fixture()
def shards(tmp_path):
    rng = np.random.default_rng(0)
    for i, n in enumerate((1000, 777, 1203)):
        np.save(tmp_path / f"edufineweb_train_{i:06d}.npy", rng.integers(0, 50257, n).astype(np.uint16))
    np.save(tmp_path / "edufineweb_val_000000.npy", rng.integers(0, 50257, 640).astype(np.uint16))
    return str(tmp_path)


@pytest.mark.parametrize("world", [1, 2, 3])
def test_windows_match_reference(shards, world):
    B, T, n = 2, 24, 40
    for rank in range(world):
        want = OD.windows(shards, "train", B, T, rank, world, n)
        ld = DataLoaderLite(B, T, rank, world, "train", data_root=shards)
        for i, (wx, wy) in enumerate(want):
            x, y = ld.next_batch()
            assert x.dtype == torch.int64 and tuple(x.shape) == (B, T)
            np.testing.assert_array_equal(x.numpy(), wx, err_msg=f"rank {rank} batch {i}")
            np.testing.assert_array_equal(y.numpy(), wy)


def test_reset_and_val_split(shards):
    ld = DataLoaderLite(4, 16, 0, 1, "val", data_root=shards)
    a = [ld.next_batch()[0].clone() for _ in range(5)]
    ld.reset()
    b = [ld.next_batch()[0].clone() for _ in range(5)]
    for u, v in zip(a, b):
        assert torch.equal(u, v)
    want = OD.windows(shards, "val", 4, 16, 0, 1, 5)
    np.testing.assert_array_equal(a[3].numpy(), want[3][0])


def test_get_most_likely_row():
    g = torch.Generator().manual_seed(0)
    E, T, V = 4, 12, 50
    tokens = torch.randint(0, V, (E, T), generator=g)
    mask = torch.zeros(E, T)
    mask[:, 5:] = 1
    mask[2, 9:] = 0
    logits = torch.randn(E, T, V, generator=g)
    logits[1, 4:11].scatter_(1, tokens[1, 5:12].unsqueeze(1), 9.0)  # ending 1 is likely
    losses = []
    for e in range(E):
        lp = torch.log_softmax(logits[e, :-1].double(), -1)
        nll = -lp.gather(1, tokens[e, 1:].unsqueeze(1)).squeeze(1)
        m = mask[e, 1:].double()
        losses.append(float((nll * m).sum() / m.sum()))
    assert get_most_likely_row(tokens, mask, logits) == int(np.argmin(losses)) == 1

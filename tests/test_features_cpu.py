"""CLIP feature shards: the reference's on-disk format
(index.json [{shard, row}] + torch.save'd [rows, L, D] shards, gpt2_linear/data.py:25-28,
56-62), written by gvl.features.FeatureShardWriter and read back per sample exactly as the
reference's CocoClipFullTokensDataset does; caption encoding vs the oracle restatement."""
import json
import os

import torch

from oracle import ops as O


def test_writer_reader_round_trip(tmp_path):
    from gvl.features import FeatureShardWriter, FeatureShards
    g = torch.Generator().manual_seed(0)
    feats = [torch.randn(n, 257, 16, generator=g) for n in (5, 7, 3)]
    w = FeatureShardWriter(str(tmp_path), rows_per_shard=4, dtype=torch.float32)
    for f in feats:
        w.add(f)
    assert w.close() == 15
    allf = torch.cat(feats)
    with open(tmp_path / "index.json") as f:
        index = json.load(f)
    assert len(index) == 15 and set(index[0]) == {"shard", "row"}
    assert [e["row"] for e in index[:5]] == [0, 1, 2, 3, 0]
    assert len({e["shard"] for e in index}) == 4  # 4 + 4 + 4 + 3 rows
    # the reference's own lookup (torch.load of the entry's shard, row r)
    for i, e in enumerate(index):
        t = torch.load(os.path.join(tmp_path, e["shard"]), map_location="cpu", weights_only=True)
        assert torch.equal(t[e["row"]], allf[i])
    r = FeatureShards(str(tmp_path))
    assert len(r) == 15
    for i in (0, 3, 4, 14, 7):
        assert torch.equal(r[i], allf[i])
    idx = [14, 0, 5, 9, 4]
    assert torch.equal(r.gather(idx), allf[idx])


def test_reader_accepts_reference_written_shards(tmp_path):
    """Shards saved by plain torch.save (the reference's precompute), legacy serialisation
    included, with an index the reference wrote (arbitrary shard names and row order)."""
    from gvl.features import FeatureShards
    a, b = torch.randn(3, 257, 8), torch.randn(2, 257, 8)
    torch.save(a, tmp_path / "train_000.pt")
    torch.save(b, tmp_path / "train_001.pt", _use_new_zipfile_serialization=False)
    index = [{"shard": "train_001.pt", "row": 1}, {"shard": "train_000.pt", "row": 2},
             {"shard": "train_000.pt", "row": 0}]
    with open(tmp_path / "index.json", "w") as f:
        json.dump(index, f)
    r = FeatureShards(str(tmp_path))
    assert torch.equal(r[0], b[1]) and torch.equal(r[1], a[2]) and torch.equal(r[2], a[0])


def test_caption_dataset_encoding_matches_reference_rule(tmp_path):
    from gvl.features import CaptionFeatureDataset, FeatureShardWriter, encode_caption
    for ids in ([], [5], list(range(40)), list(range(31)), list(range(7))):
        x, y, m = encode_caption(ids, 32, 50256)
        rx, ry, rm = O.encode_caption(ids, 32, 50256)
        assert torch.equal(x, torch.as_tensor(rx)) and torch.equal(y, torch.as_tensor(ry))
        assert torch.equal(m, torch.as_tensor(rm))
    w = FeatureShardWriter(str(tmp_path), rows_per_shard=2)
    w.add(torch.randn(3, 257, 8))
    w.close()
    caps = [[[1, 2, 3]], [[4, 5], [6]], [[7] * 50]]
    ds = CaptionFeatureDataset(str(tmp_path), caps, max_len=32, eot=99, seed=0)
    x, y, m, z = ds[2]
    assert x.shape == (31,) and z.shape == (257, 8) and z.dtype == torch.float16
    assert int(m.sum()) == 31 and int(y[-1]) == 99

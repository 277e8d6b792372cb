"""Typed mesh partials (parallel/collectives.py): device Row blocks."""
import numpy as np


def test_row_block_partial_roundtrip_matches_host_rows():
    """A rank's Row partial as device result containers (ops/device.DeviceRowBlock,
    here CPU tensors): encode_row_block -> decode_partial == the Row the host
    materialisation builds, including a Shift spill block and empty shards."""
    import torch

    from pilosa_amd import shardwidth
    from pilosa_amd.ops.device import DeviceRowBlock, GpuEngine
    from pilosa_amd.ops.gpu_executor import row_from_bitmaps
    from pilosa_amd.parallel.collectives import decode_partial, encode_row_block

    rng = np.random.default_rng(3)

    def block(shards):
        S = len(shards)
        counts = np.zeros(S * 16, np.int32)
        pay = []
        offs = np.zeros(S * 16, np.int64)
        o = 0
        for i in range(S * 16):
            kind = rng.integers(0, 3)
            if kind == 0:
                continue
            if kind == 1:
                vals = np.sort(rng.choice(65536, size=int(rng.integers(1, 300)), replace=False)).astype(np.uint16)
                n = len(vals)
                words = np.zeros((n + 7) // 8 * 8, np.uint16)
                words[:n] = vals
            else:
                bits = rng.random(65536) < 0.3
                n = int(bits.sum())
                words = np.packbits(bits, bitorder="little").view(np.uint16)
            counts[i] = n
            offs[i] = o
            pay.append(words)
            o += len(words)
        payload = np.concatenate(pay) if pay else np.zeros(8, np.uint16)
        return DeviceRowBlock(shards, torch.from_numpy(counts), torch.from_numpy(offs),
                              torch.from_numpy(payload.view(np.int16).copy()))

    M = shardwidth.DEVICE_SUBSHARDS
    main = block([0, 1, 5])
    main.spill = block([0, 5])
    w = encode_row_block(main, "cpu")
    got = decode_partial(w.numpy())

    def host(b):
        c, o, p = b.host()
        return GpuEngine.block_bitmaps(b.shards, c, o, p), b.shards
    want = row_from_bitmaps(*host(main), *host(main.spill))
    assert sorted(got.segments) == sorted(want.segments)
    assert {M, 5 + M} <= set(want.segments)     # the spill blocks landed on the next shards
    assert list(got.columns()) == list(want.columns()) and len(list(want.columns())) > 0

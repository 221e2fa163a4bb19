"""GPU radix sorts -- reduce-then-scan ("radix", csrc/hip/sort.hip) and
onesweep ("onesweep", csrc/hip/radix.hip) -- and the merge sort: exact against torch.sort for
every key type, tile-boundary sizes, skewed digit distributions (all keys
equal: one digit run per pass; sorted / reversed inputs: look-back chains of
one digit), key-value stability, bit-limited sorts, misaligned views, and
HIP-graph capture (two replays). Parity: the hw4 radix sort
(hw/hw4/programming/radixsort.cpp:22-121) checked there with std::sort."""
import pytest
import torch

from cme213x.ops.scan import lookback_timed_out
from cme213x.ops.sort import sort

TILE = 8192


def _keys(n, dtype, kind, seed=0):
    g = torch.Generator().manual_seed(seed)
    if kind == "equal":
        base = torch.full((n,), 12345, dtype=torch.int64)
    elif kind == "sorted":
        base = torch.arange(n, dtype=torch.int64) * 7919 - n
    elif kind == "reversed":
        base = -(torch.arange(n, dtype=torch.int64) * 7919 - n)
    elif kind == "fewbits":
        base = torch.randint(0, 16, (n,), generator=g, dtype=torch.int64) << 20
    else:
        base = torch.randint(-2**31, 2**31 - 1, (n,), generator=g, dtype=torch.int64)
    if dtype == torch.float32:
        x = torch.randn(n, generator=g) * 1e3 if kind == "random" else base.to(torch.float32)
        if kind == "random" and n > 10:
            x[::97] = 0.0
            x[1::97] = -0.0
            x[2::97] = float("inf")
            x[3::97] = float("-inf")
        return x
    if dtype == torch.uint32:
        return (base & 0xFFFFFFFF).to(torch.int64)
    return base.to(torch.int32)


def _to_gpu(x, dtype, dev):
    if dtype == torch.uint32:  # held as int64 in [0, 2^32) on the host (torch.sort has no uint32 kernel)
        return (x - (x >= 2**31).to(torch.int64) * 2**32).to(torch.int32).view(torch.uint32).to(dev)
    return x.to(dev)


def _from_gpu(y, dtype):
    if dtype == torch.uint32:
        y = y.view(torch.int32).cpu().to(torch.int64)
        return y + (y < 0).to(torch.int64) * 2**32
    return y.cpu()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 1000, TILE - 1, TILE, TILE + 1, 5 * TILE + 17, 1_000_003, 4 * 1024 * 1024 + 3])
@pytest.mark.parametrize("dtype", [torch.int32, torch.uint32, torch.float32])
@pytest.mark.parametrize("algo", ["radix", "onesweep"])
def test_onesweep_random(gpu, algo, n, dtype):
    x = _keys(n, dtype, "random", seed=n)
    y = _from_gpu(sort(_to_gpu(x, dtype, gpu), algo=algo), dtype)
    assert torch.equal(y, torch.sort(x).values)
    assert not lookback_timed_out(gpu)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["equal", "sorted", "reversed", "fewbits"])
@pytest.mark.parametrize("dtype", [torch.int32, torch.float32])
@pytest.mark.parametrize("algo", ["radix", "onesweep"])
def test_onesweep_skewed(gpu, algo, kind, dtype):
    n = 3 * 1024 * 1024 + 5
    x = _keys(n, dtype, kind)
    y = sort(x.to(gpu), algo=algo).cpu()
    assert torch.equal(y, torch.sort(x).values)
    assert not lookback_timed_out(gpu)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [777, 2_000_001])
@pytest.mark.parametrize("algo", ["radix", "onesweep"])
def test_onesweep_key_value_stable(gpu, algo, n):
    k = torch.randint(0, 300, (n,), dtype=torch.int32)  # long equal-key runs across tiles
    v = torch.arange(n, dtype=torch.int32)
    ks, vs = sort(k.to(gpu), v.to(gpu), algo=algo)
    ref = torch.sort(k, stable=True)
    assert torch.equal(ks.cpu(), ref.values) and torch.equal(vs.cpu(), ref.indices.to(torch.int32))
    f = torch.randn(n)
    fs, fv = sort(f.to(gpu), v.to(gpu), algo=algo)
    ref = torch.sort(f, stable=True)
    assert torch.equal(fs.cpu(), ref.values) and torch.equal(fv.cpu(), ref.indices.to(torch.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [1, 8, 12, 20, 31])
@pytest.mark.parametrize("algo", ["radix", "onesweep"])
def test_onesweep_key_bits(gpu, algo, bits):
    n = 600_001
    k = torch.randint(0, 2**bits, (n,), dtype=torch.int64).to(torch.int32)
    v = torch.arange(n, dtype=torch.int32)
    ks, vs = sort(k.to(gpu), v.to(gpu), key_bits=bits, algo=algo)
    ref = torch.sort(k, stable=True)
    assert torch.equal(ks.cpu(), ref.values) and torch.equal(vs.cpu(), ref.indices.to(torch.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["radix", "onesweep"])
def test_onesweep_misaligned_view_and_input_untouched(gpu, algo):
    x = torch.randint(-2**31, 2**31 - 1, (100_003,), dtype=torch.int32).to(gpu)
    before = x.clone()
    y = sort(x[1:], algo=algo)  # 4-byte offset: the histogram pass must not use 16-B loads
    assert torch.equal(y.cpu(), torch.sort(before[1:].cpu()).values)
    assert torch.equal(x, before)


@pytest.mark.gpu
def test_onesweep_many_calls_and_algos_agree(gpu):
    """Epoch-tagged workspace reused across calls (no memset): 30 calls of
    varying sizes, each checked; the onesweep algorithm agrees."""
    for i in range(30):
        n = 1 + (i * 37_313) % 300_000
        x = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, generator=torch.Generator().manual_seed(i))
        xg = x.to(gpu)
        a = sort(xg)
        b = sort(xg, algo="onesweep")
        assert torch.equal(a, b)
        assert torch.equal(a.cpu(), torch.sort(x).values)


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["radix", "onesweep"])
def test_onesweep_graph_capture(gpu, algo):
    n = 1_234_567
    x = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32).to(gpu)
    sort(x, algo=algo)  # warm-up outside capture
    s = torch.cuda.Stream(gpu)
    s.wait_stream(torch.cuda.current_stream(gpu))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        y = sort(x, algo=algo)
    for seed in (1, 2):
        x.copy_(torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, generator=torch.Generator().manual_seed(seed)))
        g.replay()
        torch.cuda.synchronize(gpu)
        assert torch.equal(y.cpu(), torch.sort(x.cpu()).values)


# ---------------------------------------------------------------- merge sort
MS_TILE = 4096


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 17, MS_TILE - 1, MS_TILE, MS_TILE + 1, 2 * MS_TILE - 1, 2 * MS_TILE + 1, 3 * MS_TILE + 5, 8 * MS_TILE,
                               1_000_003, 5 * 1024 * 1024 + 7])
@pytest.mark.parametrize("dtype", [torch.int32, torch.uint32, torch.float32])
def test_merge_sort_sizes(gpu, n, dtype):
    """Block sort + LDS merge-path passes (csrc/hip/sort.hip cme_merge_sort):
    partial tiles, a last run without a partner, odd and even pass counts."""
    x = _keys(n, dtype, "random", seed=n + 1)
    y = _from_gpu(sort(_to_gpu(x, dtype, gpu), algo="merge"), dtype)
    assert torch.equal(y, torch.sort(x).values)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["equal", "sorted", "reversed", "fewbits"])
def test_merge_sort_skewed_and_stable(gpu, kind):
    n = 2 * 1024 * 1024 + 3
    k = _keys(n, torch.int32, kind)
    v = torch.arange(n, dtype=torch.int32)
    ks, vs = sort(k.to(gpu), v.to(gpu), algo="merge")
    ref = torch.sort(k, stable=True)
    assert torch.equal(ks.cpu(), ref.values) and torch.equal(vs.cpu(), ref.indices.to(torch.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("part,tile,samples", [(-1, 4096, 1), (0, 4096, 1), (4, 4096, 1), (8, 4096, 1), (8, 4096, 0),
                                                (16, 4096, 1), (64, 4096, 1), (8, 8192, 1), (8, 8192, 0),
                                                (64, 8192, 1)])
def test_merge_sort_partition_arms(gpu, part, tile, samples):
    """Every way a merge pass finds its tile splits (tuning knob merge_part:
    G = 4 / 8 / 16 / 64 lanes per tile in one partition launch per pass; 0 each
    block's cooperative search; -1 the size rule), with and without the run
    samples that narrow the search to one tile first (merge_samples), and both
    merge tiles (merge_tile) sort keys and key-value pairs stably, across pair
    ends, a last run without a partner and passes of several search rounds."""
    from cme213x.utils import tuning

    g = torch.Generator(device="cuda").manual_seed(9)
    with tuning.override(merge_part=part, merge_tile=tile, merge_samples=samples):
        for n in (8193, 3 * 8192 + 4095, 1 << 20, 9 * (1 << 20) + 5):
            k = torch.randint(-(1 << 31), (1 << 31) - 1, (n,), device="cuda", dtype=torch.int32, generator=g)
            k[n // 2:] = k[n // 2:] % 11  # long runs of equal keys: ties across the split diagonals
            v = torch.arange(n, device="cuda", dtype=torch.int32)
            ks, vs = sort(k, values=v, algo="merge")
            rk, ri = torch.sort(k.cpu().long(), stable=True)
            assert torch.equal(ks.cpu().long(), rk), n
            assert torch.equal(vs.cpu().long(), ri), n
            assert torch.equal(sort(k, algo="merge").cpu().long(), rk), n


@pytest.mark.gpu
@pytest.mark.parametrize("part,samples,block", [(8, 1, 0), (8, 0, 8192), (64, 1, 16384), (4, 1, 8192)])
def test_merge_sort_four_way_passes(gpu, tune_lib, part, samples, block):
    """4-way merge passes (csrc/hip_tune/sort_tune.hip
    ms_partition4_kernel + ms_merge4_pass_kernel) sort keys and key-value
    pairs stably: groups of four runs, three (D empty), two and one at the
    array's end, an odd number of doublings (a last 2-way pass), ties across
    every run boundary, and all-equal / presorted / reversed inputs. The
    4-way schedule is a tuning-library arm (cme_merge_sort4_tune)."""
    from cme213x import _ext
    from cme213x.utils import tuning

    _ext.proto(_ext.TUNE_PROTOS, "cme_merge_sort4_tune", "ppppppqipp")
    modes = {torch.uint32: 0, torch.int32: 1, torch.float32: 2}

    def sort(k, values=None, algo="merge"):  # the 4-way arm with ops.sort's calling convention
        k = k.contiguous()
        out, tmp = torch.empty_like(k), torch.empty_like(k)
        vp = vo = vt = None
        if values is not None:
            vout, vtmp = torch.empty_like(values), torch.empty_like(values)
            vp, vo, vt = values.data_ptr(), vout.data_ptr(), vtmp.data_ptr()
        ws = torch.empty((k.numel() + 4095) // 4096 * 48 + 256, dtype=torch.uint8, device=k.device)
        _ext.call_hip("cme_merge_sort4_tune", k.data_ptr(), out.data_ptr(), tmp.data_ptr(), vp, vo, vt, k.numel(),
                      modes[k.dtype], ws.data_ptr(), _ext.stream_ptr(k.device))
        return (out, vout) if values is not None else out

    g = torch.Generator(device="cuda").manual_seed(21)
    sizes = (8193, 3 * 8192 + 5, 5 * 8192, 16 * 8192 + 4095, 17 * 16384 + 1, 3 * (1 << 20) + 77, 9 * (1 << 20) + 5)
    with tuning.override(merge_part=part, merge_samples=samples, merge_block=block):
        for n in sizes:
            k = torch.randint(-(1 << 31), (1 << 31) - 1, (n,), device="cuda", dtype=torch.int32, generator=g)
            k[n // 2:] = k[n // 2:] % 13  # long runs of equal keys
            v = torch.arange(n, device="cuda", dtype=torch.int32)
            ks, vs = sort(k, values=v, algo="merge")
            rk, ri = torch.sort(k.cpu().long(), stable=True)
            assert torch.equal(ks.cpu().long(), rk), n
            assert torch.equal(vs.cpu().long(), ri), n
            assert torch.equal(sort(k, algo="merge").cpu().long(), rk), n
        n = 3 * (1 << 20) + 11
        for kind in ("equal", "sorted", "reversed", "fewbits"):
            k = _keys(n, torch.int32, kind).to(gpu)
            v = torch.arange(n, device="cuda", dtype=torch.int32)
            ks, vs = sort(k, values=v, algo="merge")
            ref = torch.sort(k.cpu(), stable=True)
            assert torch.equal(ks.cpu(), ref.values), kind
            assert torch.equal(vs.cpu(), ref.indices.to(torch.int32)), kind
        x = torch.randn(5 * (1 << 20) + 3, device="cuda", generator=g)
        assert torch.equal(sort(x, algo="merge").cpu(), torch.sort(x.cpu()).values)


@pytest.mark.gpu
@pytest.mark.parametrize("block_sort,block", [(0, 16384), (1, 16384), (1, 32768)])
@pytest.mark.parametrize("dtype", [torch.int32, torch.float32, torch.uint32])
def test_merge_sort_radix_block_sort(gpu, block_sort, block, dtype):
    """Keys-only merge sorts from 4M keys start from 16384-key block sorts:
    the LDS radix block sort (tuning knob merge_block_sort=1, csrc/hip/sort.hip
    ms_block_radix_kernel; also with 32768-key tiles) or the merge-network
    one (0). Both give torch.sort's
    keys for int32 / float32 (signed zeros, infinities) / uint32 codes, full
    and partial tiles, one tile, and heavy duplicates."""
    from cme213x.utils import tuning

    g = torch.Generator(device="cuda").manual_seed(31)
    with tuning.override(merge_block_sort=block_sort, merge_block=block):
        for n in (1, 16383, 16384, 16385, 32768, 32769, 5 * 16384 + 77, 4 * (1 << 20) + 9, 9 * (1 << 20)):
            if dtype == torch.float32:
                k = torch.randn(n, device="cuda", generator=g)
                k[: n // 5] = torch.round(k[: n // 5])  # duplicates and signed zeros
                if n > 8:
                    k[:4] = torch.tensor([float("inf"), float("-inf"), -0.0, 0.0], device="cuda")
                ref = torch.sort(k.cpu()).values
                out = sort(k, algo="merge").cpu()
                assert torch.equal(out.view(torch.int32), ref.view(torch.int32)) or torch.equal(out, ref), n
                continue
            k = torch.randint(-(1 << 31), (1 << 31) - 1, (n,), device="cuda", dtype=torch.int32, generator=g)
            k[n // 2:] = k[n // 2:] % 17
            if dtype == torch.uint32:
                ku = k.view(torch.uint32)
                ref = torch.sort(ku.cpu().view(torch.int32).long() & 0xFFFFFFFF).values
                assert torch.equal(sort(ku, algo="merge").cpu().view(torch.int32).long() & 0xFFFFFFFF, ref), n
            else:
                assert torch.equal(sort(k, algo="merge").cpu(), torch.sort(k.cpu()).values), n
                v = torch.arange(n, device="cuda", dtype=torch.int32)  # key-value: 8192-key radix tiles, stable
                ks, vs = sort(k, values=v, algo="merge")
                rk, ri = torch.sort(k.cpu().long(), stable=True)
                assert torch.equal(ks.cpu().long(), rk) and torch.equal(vs.cpu().long(), ri), n


@pytest.mark.gpu
@pytest.mark.parametrize("block", [0, 8192, 16384])
def test_merge_sort_block_tiles(gpu, block):
    """Both block-sort tiles (tuning knob merge_block: 512 or 1024 lanes, or
    the size rule)
    sort keys and key-value pairs stably, with odd and even merge-pass counts
    and partial last tiles."""
    from cme213x.utils import tuning

    g = torch.Generator(device="cuda").manual_seed(13)
    with tuning.override(merge_block=block):
        for n in (1, 100, 16383, 16385, 3 * 16384 + 7, 1 << 20, 9 * (1 << 20) + 3):
            k = torch.randint(-(1 << 31), (1 << 31) - 1, (n,), device="cuda", dtype=torch.int32, generator=g)
            k[: n // 3] = k[: n // 3] % 5
            v = torch.arange(n, device="cuda", dtype=torch.int32)
            ks, vs = sort(k, values=v, algo="merge")
            rk, ri = torch.sort(k.cpu().long(), stable=True)
            assert torch.equal(ks.cpu().long(), rk), n
            assert torch.equal(vs.cpu().long(), ri), n
            assert torch.equal(sort(k, algo="merge").cpu().long(), rk), n


@pytest.mark.gpu
@pytest.mark.parametrize("arm", [0, 1, 2, 3, 4, 5, 7, 8, 10, 14])
def test_radix_downsweep_arms(gpu, arm):
    """Every reduce-then-scan downsweep arm (tuning knob radix_ds: atomic
    ranks, next-tile prefetch, 8192-key tiles) sorts keys and key-value pairs
    stably -- selected in-process through the tuning table."""
    from cme213x.ops.sort import sort
    from cme213x.utils import tuning

    g = torch.Generator(device="cuda").manual_seed(5)
    with tuning.override(radix_ds=arm):
        assert tuning.get("radix_ds") == arm
        for n in (1, 4097, 1 << 20, 3 * (1 << 20) + 77):
            k = torch.randint(-(1 << 31), (1 << 31) - 1, (n,), device="cuda", dtype=torch.int32, generator=g)
            k[: n // 3] = k[: n // 3] % 7
            v = torch.arange(n, device="cuda", dtype=torch.int32)
            ks, vs = sort(k, values=v, algo="radix")
            rk, ri = torch.sort(k.cpu().long(), stable=True)
            assert torch.equal(ks.cpu().long(), rk), n
            assert torch.equal(vs.cpu().long(), ri), n
            assert torch.equal(sort(k, algo="radix").cpu().long(), rk), n
    assert not tuning.is_set("radix_ds")  # restored to the environment default


@pytest.mark.gpu
def test_radix_lane_order_probe(gpu):
    """The device passes the lane-order check the lane-atomic ranks rely on
    (benchmarks/probe_lds_atomic_order.hip measured it on gfx950), and the
    answer is cached per device."""
    from cme213x.ops.sort import radix_lane_order

    assert radix_lane_order(check=True)
    assert radix_lane_order(check=False)


@pytest.mark.gpu
@pytest.mark.parametrize("arm", [2, 10, 14])
@pytest.mark.parametrize("kind", ["equal", "sorted", "reversed", "fewbits", "small", "twovals"])
def test_radix_lane_ranks_low_entropy_stable(gpu, arm, kind):
    """Lane-atomic ranks (arm 10) against the ballot-match arm (2) and a
    stable CPU sort on inputs whose waves see one or a few digits: all keys
    equal, sorted / reversed runs, few bits, small keys (high digits all
    zero: the one-atomic-per-wave path), two values interleaved."""
    from cme213x.ops.sort import sort
    from cme213x.utils import tuning

    n = 3 * (1 << 20) + 1234
    if kind == "small":
        k = torch.randint(0, 1 << 12, (n,), dtype=torch.int32)
    elif kind == "twovals":
        k = (torch.arange(n, dtype=torch.int32) % 2) * 0x01010101
    else:
        k = _keys(n, torch.int32, kind)
    v = torch.arange(n, dtype=torch.int32)
    with tuning.override(radix_ds=arm):
        ks, vs = sort(k.to(gpu), values=v.to(gpu), algo="radix")
    ref = torch.sort(k.long(), stable=True)
    assert torch.equal(ks.cpu().long(), ref.values)
    assert torch.equal(vs.cpu().long(), ref.indices)


@pytest.mark.gpu
@pytest.mark.parametrize("values", [False, True])
def test_merge_sort_in_place_misaligned(gpu, values):
    """The in-place C entry (cme_merge_sort_u32) on arrays that start 4 B past
    a 16-B boundary: full output tiles must fall back from their 16-B stores
    (csrc/hip/sort_kernels.h ms_store_tile) instead of faulting or tearing."""
    from cme213x import _ext

    n = 3 * (1 << 20) + 5
    g = torch.Generator(device="cuda").manual_seed(41)
    buf = torch.randint(0, 2**31 - 1, (n + 1,), device="cuda", dtype=torch.int32, generator=g)
    keys = buf[1:]  # 4-B offset
    orig = keys.cpu().long()
    ref, ref_idx = torch.sort(orig, stable=True)
    alt = torch.empty(n + 1, device="cuda", dtype=torch.int32)[1:]
    vals = valt = None
    if values:
        vb = torch.arange(n + 1, device="cuda", dtype=torch.int32)
        vals = vb[1:]
        valt = torch.empty(n + 1, device="cuda", dtype=torch.int32)[1:]
    _ext.call_hip("cme_merge_sort_u32", keys.data_ptr(), alt.data_ptr(), vals.data_ptr() if values else None,
                  valt.data_ptr() if values else None, n, _ext.stream_ptr(gpu))
    torch.cuda.synchronize(gpu)
    assert torch.equal(keys.cpu().long(), ref)
    if values:  # stable: each key carries its original position (values started at 1)
        assert torch.equal(vals.cpu().long(), ref_idx + 1)

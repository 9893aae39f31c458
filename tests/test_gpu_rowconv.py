"""The register-fed forward conv with the fused rescale (niti_conv_fwd_rows, csrc/niti_rowconv.hip)
against the oracle's NITI_Conv_Int8 (NITI_Conv_Int8.cpp:162-310): requantised output, exponent,
relu, the fused 2x2 max pool and the next layer's C32 copy, bit for bit, in all three modes (fused
one-launch with the in-kernel grid barrier; range then recompute-and-requantise), on every image
width the kernel takes, ragged image groups (batch not a multiple of 32 / W) and every branch of
the shift rule (raw cast, shift == 1 -> 2, shift > 1)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def T():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import niti_amd  # noqa: F401
    return torch


def _case(T, n, ci, h, co, relu, pool, mode, seed, wmax=127, xmax=127, x_nhwc=False):
    import niti_oracle as O
    from niti_amd import ops
    rng = np.random.default_rng(seed)
    g = O.geom(n, ci, h, h, co, 3, pad=1)
    x = rng.integers(-xmax, xmax + 1, (n, ci, h, h)).astype(np.int8)
    w = rng.integers(-wmax, wmax + 1, (co, ci, 3, 3)).astype(np.int8)
    y_ref, e_ref, acc, _ = O.conv_fwd(g, x, w, -3, -5)
    r_ref = O.relu(y_ref) if relu else y_ref
    dev = lambda a: T.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    gg = ops.geom(n, ci, h, h, co, 3, pad=1)
    assert ops.conv_rows_ok(gg)
    x16 = ops.nchw_to_nhwc16(dev(x))
    xc = ops.nhwc16_to_c32(x16, ci)
    wf = ops.weights_to_wf(ops.oihw_to_ohwi16(dev(w)), ci)
    ein, ws = dev(np.array([-3], np.int8)), dev(np.array([-5], np.int8))
    eo = T.zeros(1, dtype=T.int8, device="cuda")
    amax = ops.new_range()
    st = ops.RowConvState()
    kw = dict(exp_in=ein, wscale=ws, exp_out=eo, relu=relu, pool=pool, next_c32=True)
    if x_nhwc:  # the row-segment form reading its NHWC16 input in place
        assert ops.rows_nhwc_ok(gg)
        xc = x16
        kw["x_nhwc"] = True
    def check(out, pout, nxt):
        T.cuda.synchronize()
        assert int(st.err.item()) == 0
        got = out.cpu().numpy()[..., :co].transpose(0, 3, 1, 2)
        assert np.array_equal(got, r_ref)
        assert int(eo.item()) == e_ref
        if pool:
            p_ref = O.maxpool(r_ref)
            assert np.array_equal(pout.cpu().numpy()[..., :co].transpose(0, 3, 1, 2), p_ref)
            want_next = p_ref
        else:
            want_next = r_ref
        nx = nxt.cpu().numpy()  # [n][cb][h][w][32]
        nx = nx.transpose(0, 1, 4, 2, 3).reshape(n, -1, nx.shape[2], nx.shape[3])[:, :co]
        assert np.array_equal(nx, want_next)

    if mode == 0:
        check(*ops.conv_fwd_rows(gg, xc, wf, amax, mode=0, state=st, **kw))
    elif mode == 4:
        _spec_pairs(T, st, False, amax, eo, lambda m, outs: ops.conv_fwd_rows(gg, xc, wf, amax, mode=m, state=st,
                                                                              outs=outs, **kw), check)
    else:
        ops.conv_fwd_rows(gg, xc, wf, amax, mode=1, **kw)
        check(*ops.conv_fwd_rows(gg, xc, wf, amax, mode=2, **kw))
    return int(np.abs(acc).max())


def _spec_pairs(T, st, dgrad, amax, eo, launch, check):
    """The speculative pair (modes 3 + 4) three times on one state: no hint yet (launch 4 redoes),
    the hint of the first pair (a hit: launch 4 exits at once), and a hint forced one bit wide
    (launch 4 redoes); every pair's outputs are the rule's, and the slot counts the two misses."""
    off = st.spec_offset(dgrad)
    for rep in range(3):
        if rep == 2:  # every predictor's next guess one bit wide (spec_pick: words 0 / 24 / 25)
            for j in (0, 24, 25):
                hint = int(st.state[off + j].item())
                if hint != 0:
                    st.state[off + j] = hint + 1
        amax.zero_()
        if eo is not None:
            eo.zero_()
        outs = launch(3, None)
        outs = launch(4, outs)
        check(*outs)
        assert st.spec_slot(dgrad)[2] == (1 if rep < 2 else 2), (rep, st.spec_slot(dgrad))


@pytest.mark.parametrize("h", [2, 4, 8, 16])
@pytest.mark.parametrize("mode", [0, 2, 4])
def test_rows_fwd_widths(T, h, mode):
    for k, (n, ci, co, relu, pool) in enumerate([(3, 32, 32, True, True), (17, 64, 64, False, False),
                                                  (1, 96, 32, True, False), (8, 32, 96, False, True)]):
        if pool and h < 2:
            continue
        _case(T, n, ci, h, co, relu, pool, mode, seed=100 * h + 10 * mode + k)


def test_rows_fwd_shift_branches(T):
    """Small operands drive max|acc| through the raw-cast (bw <= 7), shift == 1 (bw == 8) and
    shift > 1 branches of the rule (NITI_Conv_Int8.cpp:266-307)."""
    seen = set()
    for seed, (wmax, xmax) in enumerate([(1, 1), (1, 2), (1, 3), (2, 2), (2, 3), (3, 4), (127, 127)]):
        for mode in (0, 2, 4):
            m = _case(T, 4, 32, 4, 32, False, False, mode, seed=900 + seed, wmax=wmax, xmax=xmax)
            bw = 0 if m <= 1 else int(np.ceil(np.log2(m)))
            seen.add("raw" if bw <= 7 else "one" if bw == 8 else "psto")
    assert seen == {"raw", "one", "psto"}


def test_rows_fwd_vgg11_conv4_shape(T):
    """The headline layer's shape (VGG-11 conv4: 256 -> 256 at 8x8) at batch 32, fused launch."""
    _case(T, 32, 256, 8, 256, True, True, 0, seed=4)


def _dgrad_case(T, n, ci, h, co, pool, relu, mode, seed, wmax=127, dmax=127, p16=True, x_nhwc=False):
    """The layer (ci -> co at h x h) input gradient on the row kernel against NITI's dgrad
    (NITI_DeConv_Int8.cpp:294-329 requantised by the forward rule) followed by the previous
    layer's relu gradient (NITI_ReluGrad_Int8) or its 2x2 max-pool + relu gradient
    (NITI_CPUPoolGrad_Int8, maxpool_relu_grad)."""
    import niti_oracle as O
    from niti_amd import ops
    rng = np.random.default_rng(seed)
    g = O.geom(n, ci, h, h, co, 3, pad=1)
    dy = rng.integers(-dmax, dmax + 1, (n, co, h, h)).astype(np.int8)
    w = rng.integers(-wmax, wmax + 1, (co, ci, 3, 3)).astype(np.int8)
    dq, _, acc, _ = O.conv_dgrad(g, dy, w)
    dev = lambda a: T.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    nhwc = lambda a: ops.nchw_to_nhwc16(dev(a))  # noqa: E731
    if pool:
        px = rng.integers(-2, 6, (n, ci, 2 * h, 2 * h)).astype(np.int8)  # ties and non-positives
        if relu:
            px = np.maximum(px, 0).astype(np.int8)
        py = O.maxpool(px)
        want = O.maxpool_grad(px, py, dq)
        if relu:
            want = O.relu_grad(px, want)
    else:
        mk = rng.integers(-2, 3, (n, ci, h, h)).astype(np.int8)
        want = O.relu_grad(mk, dq) if relu else dq
    gg = ops.geom(n, ci, h, h, co, 3, pad=1)
    dyc = ops.nhwc16_to_c32(nhwc(dy), co)
    wft = ops.weights_to_wf(ops.oihw_to_ohwi16(dev(w)), ci, transpose=True)
    amax = ops.new_range()
    st = ops.RowConvState()
    kw = dict(dx_c32=True, dx_p16=p16)
    if x_nhwc:  # dy NHWC16 read in place
        assert ops.rows_nhwc_ok(gg, dgrad=True)
        dyc = nhwc(dy)
        kw["x_nhwc"] = True
    if pool:
        kw.update(pool_x=nhwc(px), pool_y=nhwc(py), pool_relu=relu)
    elif relu:
        kw.update(relu_mask=nhwc(mk))
    from niti_amd._lib import NitiError

    def launch(**k):
        if mode == 0:
            return ops.conv_dgrad_rows(gg, dyc, wft, amax, mode=0, state=st, **k)
        if mode == 4:  # the pair's first call here (the NOT_SUPPORT probe); _spec_pairs repeats it
            outs = ops.conv_dgrad_rows(gg, dyc, wft, amax, mode=3, state=st, **k)
            return ops.conv_dgrad_rows(gg, dyc, wft, amax, mode=4, state=st, outs=outs, **k)
        ops.conv_dgrad_rows(gg, dyc, wft, amax, mode=1, **k)
        return ops.conv_dgrad_rows(gg, dyc, wft, amax, mode=2, **k)

    def check(dx, dxc, p16):
        T.cuda.synchronize()
        assert int(st.err.item()) == 0
        assert np.array_equal(dx.cpu().numpy()[..., :ci].transpose(0, 3, 1, 2), want)
        nx = dxc.cpu().numpy()
        nx = nx.transpose(0, 1, 4, 2, 3).reshape(n, -1, nx.shape[2], nx.shape[3])[:, :ci]
        assert np.array_equal(nx, want)
        if p16 is not None:  # the weight gradient's pixel blocks, as niti_nhwc16_to_p16 lays them out
            assert np.array_equal(p16.cpu().numpy(), ops.nhwc16_to_p16(dx).cpu().numpy())

    try:
        res = launch(**kw)
    except NitiError as e:  # no whole 16-pixel blocks per wave (4x4 images, no pool, small batch) or tensor
        assert e.code == 2 and not pool and (h == 4 or n * h * h % 16 != 0), (e, h, pool)
        kw["dx_p16"] = False
        res = launch(**kw)
    if mode == 4:
        st.state.zero_()  # a fresh slot for the three pairs
        _spec_pairs(T, st, True, amax, None, lambda m, outs: ops.conv_dgrad_rows(gg, dyc, wft, amax, mode=m, state=st,
                                                                                 outs=outs, **kw), check)
    else:
        check(*res)
    return int(np.abs(acc).max())


@pytest.mark.parametrize("h", [2, 4, 8, 16])
@pytest.mark.parametrize("mode", [0, 2, 4])
def test_rows_dgrad_widths(T, h, mode):
    for k, (n, ci, co, pool, relu) in enumerate([(3, 32, 32, True, True), (17, 64, 64, False, True),
                                                  (1, 96, 32, True, False), (8, 32, 96, False, False)]):
        _dgrad_case(T, n, ci, h, co, pool, relu, mode, seed=500 + 100 * h + 10 * mode + k)


def test_rows_dgrad_shift_branches(T):
    seen = set()
    for seed, (wmax, dmax) in enumerate([(1, 1), (1, 2), (1, 3), (2, 2), (2, 3), (3, 4), (127, 127)]):
        m = _dgrad_case(T, 4, 32, 4, 32, seed % 2 == 0, True, seed % 2, seed=700 + seed, wmax=wmax, dmax=dmax)
        bw = 0 if m <= 1 else int(np.ceil(np.log2(m)))
        seen.add("raw" if bw <= 7 else "one" if bw == 8 else "psto")
    assert seen == {"raw", "one", "psto"}


def test_rows_dgrad_vgg11_shapes(T):
    """VGG-11's input gradients at batch 32: conv4 (256 -> 512 at 4x4, into conv3's pool) and
    conv2 (128 -> 256 at 8x8, into conv1's pool), fused launches."""
    _dgrad_case(T, 32, 256, 4, 512, True, True, 0, seed=41)
    _dgrad_case(T, 32, 256, 8, 256, False, True, 0, seed=42)


@pytest.mark.parametrize("mode", [0, 2, 4])
def test_rows_ks_2x2(T, mode):
    """The K-split form (rowconv_compute_ks: 2x2 maps whose conv input channels are a multiple of
    128 -- one unit per workgroup, the four waves splitting the channel chunks, partial tiles summed
    through LDS), forward and input gradient, ragged batches, 1 / 2 / 4 chunks per wave."""
    for k, (n, ci, co, relu, pool) in enumerate([(17, 128, 32, True, True), (33, 256, 64, False, False),
                                                  (40, 512, 96, True, False), (16, 512, 512, True, True)]):
        _case(T, n, ci, 2, co, relu, pool, mode, seed=900 + 10 * mode + k)
    for k, (n, ci, co, pool, relu) in enumerate([(17, 32, 128, True, True), (33, 64, 256, False, True),
                                                  (40, 96, 512, True, False), (16, 512, 512, False, False)]):
        _dgrad_case(T, n, ci, 2, co, pool, relu, mode, seed=950 + 10 * mode + k)


def test_rows_ks_vgg11_2x2_b256(T):
    """VGG-11's 2x2 layers at the benchmarked batch (512 -> 512, 256 images: 256 K-split
    workgroups), fused launches: conv7's forward with its pool and conv8's input gradient into
    conv7's relu."""
    _case(T, 256, 512, 2, 512, True, True, 0, seed=31)
    _dgrad_case(T, 256, 512, 2, 512, False, True, 0, seed=32)


# ---- the row-segment form (W = 0): maps of 14 / 28 / 56 / 112 / 224 px as 14-px segments with halo
# lanes (one 14-px row of two images at 14 px) -- VGG-16's and ResNet-18's stride-1 3x3 layers


@pytest.mark.parametrize("h", [14, 28, 56])
@pytest.mark.parametrize("mode", [0, 2, 4])
def test_rows_seg_fwd(T, h, mode):
    """Forward with the rescale (fused launch, or range then recompute-and-requantise), relu, the
    2x2 pool (pairs inside a segment) and the C32 copy, ragged image pairs at 14 px."""
    for k, (n, ci, co, relu, pool) in enumerate([(2, 32, 32, True, True), (3, 64, 96, False, False),
                                                  (1, 96, 64, True, True)]):
        _case(T, n, ci, h, co, relu, pool, mode, seed=2000 + 100 * h + 10 * mode + k)


@pytest.mark.parametrize("h", [112, 224])
def test_rows_seg_fwd_large(T, h):
    _case(T, 1, 32, h, 32, True, True, 2, seed=3000 + h)
    _case(T, 2, 64, h, 32, False, False, 0, seed=3001 + h)


@pytest.mark.parametrize("h", [14, 28, 56])
@pytest.mark.parametrize("mode", [0, 2, 4])
def test_rows_seg_dgrad(T, h, mode):
    """Input gradient on the row-segment form with the previous layer's relu gradient or its 2x2
    max-pool (+ relu) gradient routed into the full-resolution map, NHWC16 and C32 outputs."""
    for k, (n, ci, co, pool, relu) in enumerate([(2, 32, 32, True, True), (3, 64, 96, False, True),
                                                  (1, 96, 64, True, False), (2, 32, 64, False, False)]):
        _dgrad_case(T, n, ci, h, co, pool, relu, mode, seed=4000 + 100 * h + 10 * mode + k, p16=False)


def test_rows_seg_shift_branches(T):
    seen = set()
    for seed, (wmax, xmax) in enumerate([(1, 1), (1, 2), (1, 3), (2, 3), (3, 4), (127, 127)]):
        for mode in (0, 2, 4):
            m = _case(T, 2, 32, 28, 32, False, False, mode, seed=5000 + seed, wmax=wmax, xmax=xmax)
            bw = 0 if m <= 1 else int(np.ceil(np.log2(m)))
            seen.add("raw" if bw <= 7 else "one" if bw == 8 else "psto")
    assert seen == {"raw", "one", "psto"}


@pytest.mark.parametrize("h", [14, 28, 56])
@pytest.mark.parametrize("mode", [0, 2, 4])
def test_rows_seg_nhwc_input(T, h, mode):
    """The row-segment form reading its input (x, or dy) as NHWC16 in place (NITI_ROWS_X_NHWC16):
    the same outputs as from the C32 copy, forward and input gradient."""
    for k, (n, ci, co, relu, pool) in enumerate([(2, 32, 32, True, True), (3, 64, 96, False, False),
                                                  (1, 96, 64, True, True)]):
        _case(T, n, ci, h, co, relu, pool, mode, seed=6000 + 100 * h + 10 * mode + k, x_nhwc=True)
    for k, (n, ci, co, pool, relu) in enumerate([(2, 32, 32, True, True), (3, 64, 96, False, True),
                                                  (1, 96, 64, True, False)]):
        _dgrad_case(T, n, ci, h, co, pool, relu, mode, seed=6500 + 100 * h + 10 * mode + k, p16=False, x_nhwc=True)


def test_rows_seg_nhwc_input_large(T):
    _case(T, 2, 64, 112, 64, True, True, 2, seed=6901, x_nhwc=True)
    _dgrad_case(T, 1, 64, 224, 64, False, True, 2, seed=6902, p16=False, x_nhwc=True)

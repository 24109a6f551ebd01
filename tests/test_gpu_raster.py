"""GPU parity of the gfx950 rasterizer against the CPU oracle (oracle/gs_oracle.c).

Bar (DESIGN.md "Parity"): tile/key indexing bit-exact (sorted (tile, Gaussian) list, ranges, radii,
num_rendered, precise instance count, per-Gaussian geometry); images within the exp() ulp budget
(PSNR(HIP, oracle) >= 80 dB, i.e. far inside the north-star's 1e-3 dB PSNR tolerance); gradients within
rel. L2 error 1e-4 of the oracle's restatement of the reference bucket backward."""
import numpy as np
import pytest
import torch

from raster_util import (hip_forward, hip_geometry, hip_image_state, hip_sorted_instances, oracle_forward,
                         per_tile_lists, psnr, rel_err, small_scene)

pytestmark = pytest.mark.gpu

CASES = [
    # (n, W, H, deg, bg, aa)
    (1, 64, 48, 3, (0, 0, 0), False),
    (64, 64, 48, 3, (0.1, 0.5, 0.9), False),
    (1024, 133, 97, 3, (1, 1, 1), False),
    (1024, 133, 97, 1, (0, 0, 0), True),
    (3000, 256, 192, 2, (0.2, 0.3, 0.4), False),
    (20000, 800, 800, 3, (0, 0, 0), False),
    # dense 16x12 tiles: with 2 per tile in phase 1 the phase-2 lists run to hundreds of splats, so the longest are
    # composited as segments and joined (DESIGN.md §3 Forward 6), pixels stopping inside a segment included
    (12000, 256, 192, 3, (0.2, 0.3, 0.4), False),
]


@pytest.fixture(params=[0, 2], ids=["prefix-default", "prefix-2-per-tile"])
def prefix_policy(request):
    """Depth-prefix binning: the library default, and a tiny phase-1 capacity that forces phase 2."""
    from dogs_amd.diff_gaussian_rasterization import _C
    old = _C.set_prefix_per_tile(request.param)
    yield request.param
    _C.set_prefix_per_tile(old)


@pytest.mark.parametrize("n,W,H,deg,bg,aa", CASES)
def test_forward_bitexact_keys(oracle, hip_device, prefix_policy, n, W, H, deg, bg, aa):
    s = small_scene(n, W, H, seed=7 + n)
    col_o, radii_o, inv_o, st = oracle_forward(oracle, s, bg, deg=deg, antialiasing=aa)
    out = hip_forward(s, bg, hip_device, deg=deg, antialiasing=aa)
    num_rendered, K, col, inv, radii = out[:5]
    assert num_rendered == st.num_rendered
    assert K >= 1  # the phase-1 capacity token
    np.testing.assert_array_equal(radii.cpu().numpy(), radii_o)
    # every tile's binned list is a prefix of the reference order (tile, depth bits, index) ...
    t_o, i_o, _ = st.sorted_list()
    t_h, i_h, e1 = hip_sorted_instances(out, W, H, hip_device, n)
    assert e1 <= len(t_h) <= st.num_valid
    full = per_tile_lists(t_o, i_o, len(t_o))
    got = per_tile_lists(t_h, i_h, e1)
    for t, lst in got.items():
        assert lst == full[t][:len(lst)], f"tile {t}: not a prefix of the reference list"
    fT_o, nc_o, mc_o = st.image_state()
    fT, nc, mc, rg = hip_image_state(out, W, H, hip_device)
    # ... that reaches every pixel's last contributor (and is the whole list when nothing was cut)
    T = len(st.ranges())
    tx = (W + 15) // 16
    for t in range(T):
        m = int(mc[t])
        assert m <= len(got.get(t, [])), f"tile {t}: max contributor {m} beyond its binned list"
    if e1 == st.num_valid:  # phase 1 binned everything: the whole reference order
        np.testing.assert_array_equal(t_h, t_o)
        np.testing.assert_array_equal(i_h, i_o)
        np.testing.assert_array_equal(rg, st.ranges())
    xy, co, rgbi, cnt = hip_geometry(out, n, hip_device)
    g = st.geom()
    vis = radii_o > 0
    np.testing.assert_array_equal(xy[vis], g["means2D"][vis])
    np.testing.assert_array_equal(co[vis], g["conic_opacity"][vis])
    binned = cnt > 0  # colours are evaluated for the binned Gaussians only (the others are never composited)
    assert binned[vis].any()
    np.testing.assert_array_equal(rgbi[binned, :3], g["rgb"][binned])
    # compositing: only exp() differs (v_exp_f32 vs libm expf)
    assert (nc == nc_o).mean() > 0.999
    assert psnr(col.cpu().numpy(), col_o) > 80.0
    assert psnr(inv.cpu().numpy(), inv_o) > 60.0
    assert np.abs(col.cpu().numpy() - col_o).max() < 5e-3
    del tx


def _backward_vs_oracle(s, W, H, deg, bg, aa, dev, seed):
    from dogs_amd.diff_gaussian_rasterization import _C
    col_o, radii_o, inv_o, st = oracle_forward(oracle_mod(), s, bg, deg=deg, antialiasing=aa)
    out = hip_forward(s, bg, dev, deg=deg, antialiasing=aa)
    rng = np.random.default_rng(seed)
    gcol = rng.standard_normal((3, H, W)).astype(np.float32)
    ginv = (0.1 * rng.standard_normal((1, H, W))).astype(np.float32)
    go = st.backward(gcol, ginv[0])
    c = s.camera.to(dev)
    e = torch.empty(0, device=dev)
    d = lambda t: t.to(dev).contiguous()  # noqa: E731
    gr = _C.rasterize_gaussians_backward(
        torch.as_tensor(bg, dtype=torch.float32, device=dev), d(s.means3D), out[4], e, d(s.opacities), d(s.scales),
        d(s.rotations), 1.0, e, c.world_to_camera, c.projective_matrix, c.tanfovx, c.tanfovy,
        torch.from_numpy(gcol).to(dev), d(s.dc), d(s.sh), torch.from_numpy(ginv).to(dev), deg, c.camera_center,
        out[5], out[0], out[6], out[7], out[1], out[8], aa, False)
    names = ["dmeans2D", "dcolors", "dopacity", "dmeans3D", "dcov3D", "ddc", "dsh", "dscales", "drot", "depth"]
    for name, h in zip(names, gr):
        ref = go[name]
        err = rel_err(h.cpu().numpy().reshape(ref.shape), ref)
        assert err < 1e-4, f"{name}: rel err {err}"
    return st


def oracle_mod():
    from oracle import oracle as O
    return O


@pytest.mark.parametrize("n,W,H,deg,bg,aa", CASES)
def test_backward_matches_oracle(oracle, hip_device, prefix_policy, n, W, H, deg, bg, aa):
    s = small_scene(n, W, H, seed=11 + n)
    _backward_vs_oracle(s, W, H, deg, bg, aa, hip_device, seed=n)


def test_backward_huge_splats(oracle, hip_device, prefix_policy):
    """A few splats spanning hundreds of tiles: their instance records take the whole-wave summation path
    of k_record_sum (lists longer than 256) and the wide-rect candidate walk of preprocess/emit."""
    n, W, H = 2000, 640, 480
    s = small_scene(n, W, H, seed=5)
    big = torch.arange(0, n, 97)
    s.scales[big] = s.scales[big] * 40.0
    st = _backward_vs_oracle(s, W, H, 3, (0.3, 0.2, 0.1), False, hip_device, seed=5)
    assert int(st.geom()["tiles_touched"].max()) > 256


@pytest.mark.parametrize("seed", [3, 4])
def test_tight_walk_thin_and_faint(oracle, hip_device, seed):
    """The binning walks enumerate only the tiles of the contribution ellipse's bounding box (raster_fwd.hip
    tight_rect): on needle-thin rotated splats (scales 30x and 0.03x of the scene's), faint ones around the alpha
    1/255 cut (opacity 0.5/255 .. 4/255) and opaque ones, the binned instance list must still be the reference's,
    instance for instance, with everything binned in one phase."""
    from dogs_amd.diff_gaussian_rasterization import _C
    n, W, H = 4000, 320, 240
    s = small_scene(n, W, H, seed=seed)
    g = torch.Generator().manual_seed(seed)
    thin = torch.rand(n, generator=g) < 0.5
    k = torch.ones((n, 3))
    k[thin, 0] = 30.0
    k[thin, 1] = 0.03
    s.scales = (s.scales * k).contiguous()
    faint = torch.rand(n, generator=g) < 0.3
    op = s.opacities.clone()
    op[faint, 0] = (0.5 + 3.5 * torch.rand(int(faint.sum()), generator=g)) / 255.0
    s.opacities = op.contiguous()
    old = _C.set_prefix_per_tile(-1)
    try:
        col_o, radii_o, inv_o, st = oracle_forward(oracle, s, (0, 0, 0), deg=3)
        out = hip_forward(s, (0, 0, 0), hip_device, deg=3)
        assert int(out[0]) == st.num_rendered
        t_o, i_o, _ = st.sorted_list()
        t_h, i_h, e1 = hip_sorted_instances(out, W, H, hip_device, n)
        assert e1 == len(t_h) == st.num_valid
        np.testing.assert_array_equal(t_h, t_o)
        np.testing.assert_array_equal(i_h, i_o)
        assert psnr(out[2].cpu().numpy(), col_o) > 80.0
    finally:
        _C.set_prefix_per_tile(old)


@pytest.mark.parametrize("n,W,H,mode", [(3000, 256, 192, "clones"), (600, 64, 48, "planar"),
                                        (20000, 128, 96, "dense-clones")])
@pytest.mark.parametrize("prefix", [0, 2, -1], ids=["prefix-default", "prefix-2-per-tile", "no-prefix"])
def test_equal_depth_order(oracle, hip_device, n, W, H, mode, prefix):
    """Equal view depths (cloned Gaussians, a camera-facing plane) must come out in Gaussian index order, as the
    reference's stable radix sort leaves them; 'dense' lists exceed the per-wave sort capacity (block kernel)."""
    from dogs_amd.diff_gaussian_rasterization import _C
    s = small_scene(n, W, H, seed=21)
    if mode in ("clones", "dense-clones"):  # second half: copies of the first half's depth, shifted in x/y
        h = n // 2
        s.means3D[h:2 * h, 2] = s.means3D[:h, 2]
        s.means3D[h:2 * h, :2] = s.means3D[:h, :2] * 0.97
    else:  # every Gaussian at one depth
        s.means3D[:, 2] = float(s.means3D[0, 2])
    old = _C.set_prefix_per_tile(prefix)
    try:
        col_o, radii_o, inv_o, st = oracle_forward(oracle, s, (0.1, 0.2, 0.3))
        out = hip_forward(s, (0.1, 0.2, 0.3), hip_device)
        t_o, i_o, _ = st.sorted_list()
        t_h, i_h, e1 = hip_sorted_instances(out, W, H, hip_device, n)
        full = per_tile_lists(t_o, i_o, len(t_o))
        got = per_tile_lists(t_h, i_h, e1)
        assert max(len(v) for v in full.values()) > (512 if mode == "dense-clones" else 0)
        for t, lst in got.items():
            assert lst == full[t][:len(lst)], f"tile {t}: not a prefix of the reference list"
        assert psnr(out[2].cpu().numpy(), col_o) > 80.0
    finally:
        _C.set_prefix_per_tile(old)


def test_adaptive_prefix_capacity(oracle, hip_device):
    """prefix_per_tile = 0: the phase-1 capacity grows while views leave tiles unfinished (translucent scene, phase 2
    on every early view), images do not depend on it, and a view's backward uses the capacity its forward returned
    even after later forwards grew it."""
    from dogs_amd.diff_gaussian_rasterization import _C
    n, W, H = 20000, 112, 80  # an image size no other test uses: fresh adaptive state
    s = small_scene(n, W, H, seed=31)
    s.opacities = (s.opacities * 0.05).contiguous()
    bg = (0.1, 0.2, 0.3)
    col_o, radii_o, inv_o, st = oracle_forward(oracle, s, bg)
    old = _C.set_prefix_per_tile(0)
    try:
        first = hip_forward(s, bg, hip_device)
        tokens = [int(first[1])]
        for _ in range(10):
            o = hip_forward(s, bg, hip_device)
            torch.cuda.synchronize()
            tokens.append(int(o[1]))
            assert psnr(o[2].cpu().numpy(), col_o) > 80.0
        assert tokens == sorted(tokens) and tokens[-1] > tokens[0], tokens
        # backward of the first view (small capacity, phase 2) after the capacity grew
        dev = hip_device
        c = s.camera.to(dev)
        e = torch.empty(0, device=dev)
        d = lambda t: t.to(dev).contiguous()  # noqa: E731
        rng = np.random.default_rng(3)
        gcol = rng.standard_normal((3, H, W)).astype(np.float32)
        go = st.backward(gcol)
        gr = _C.rasterize_gaussians_backward(
            torch.as_tensor(bg, dtype=torch.float32, device=dev), d(s.means3D), first[4], e, d(s.opacities),
            d(s.scales), d(s.rotations), 1.0, e, c.world_to_camera, c.projective_matrix, c.tanfovx, c.tanfovy,
            torch.from_numpy(gcol).to(dev), d(s.dc), d(s.sh), torch.zeros((1, H, W), device=dev), 3,
            c.camera_center, first[5], first[0], first[6], first[7], first[1], first[8], False, False)
        for name, h in zip(["dmeans2D", "dcolors", "dopacity", "dmeans3D"], gr):
            ref = go[name]
            assert rel_err(h.cpu().numpy().reshape(ref.shape), ref) < 1e-4, name
        assert psnr(first[2].cpu().numpy(), col_o) > 80.0
    finally:
        _C.set_prefix_per_tile(old)


def test_capacity_contexts_are_isolated(hip_device):
    """dg_raster_args.capacity_ctx: the adaptive capacity grown under one context (a translucent scene: phase 2 on every
    early view) leaves another context cold, and a view rendered cold under either context has the same capacity
    token, the same images and bit-identical gradients (the per-Gaussian sums round by instance position, so the
    rounding follows the capacity history -- which is why every trainer renders under its own context)."""
    from dogs_amd.diff_gaussian_rasterization import _C
    n, W, H = 20000, 104, 72  # an image size no other test uses
    s = small_scene(n, W, H, seed=33)
    s.opacities = (s.opacities * 0.05).contiguous()
    bg = (0.1, 0.2, 0.3)
    dev = hip_device
    c = s.camera.to(dev)
    e = torch.empty(0, device=dev)
    d = lambda t: t.to(dev).contiguous()  # noqa: E731
    gcol = torch.from_numpy(np.random.default_rng(5).standard_normal((3, H, W)).astype(np.float32)).to(dev)

    def view():
        o = hip_forward(s, bg, dev)
        g = _C.rasterize_gaussians_backward(
            torch.as_tensor(bg, dtype=torch.float32, device=dev), d(s.means3D), o[4], e, d(s.opacities), d(s.scales),
            d(s.rotations), 1.0, e, c.world_to_camera, c.projective_matrix, c.tanfovx, c.tanfovy, gcol, d(s.dc),
            d(s.sh), torch.zeros((1, H, W), device=dev), 3, c.camera_center, o[5], o[0], o[6], o[7], o[1], o[8],
            False, False)
        torch.cuda.synchronize()
        return int(o[1]), o[2].clone(), [t.clone() for t in g]

    old = _C.set_prefix_per_tile(0)
    try:
        a, b = _C.new_capacity_context(), _C.new_capacity_context()
        with _C.capacity_context(a):
            first_a = view()
            grown = [view()[0] for _ in range(8)]
        assert grown[-1] > first_a[0], "the translucent scene must grow context a's capacity"
        with _C.capacity_context(b):
            first_b = view()
        assert first_b[0] == first_a[0], "context b starts cold"
        assert torch.equal(first_b[1], first_a[1])
        for x, y in zip(first_b[2], first_a[2]):
            assert torch.equal(x, y)
        with _C.capacity_context(a):      # context a kept its growth
            assert view()[0] >= grown[-1]
        assert view()[0] == first_a[0], "the default context is untouched by both"
    finally:
        _C.set_prefix_per_tile(old)


@pytest.mark.parametrize("per_tile", [0, -1], ids=["prefix-default", "prefix-off"])
def test_forward_many_binning_waves(oracle, hip_device, per_tile):
    """More than 16384 binning waves (P > 2^20): the ranges scan runs several rounds of 16 items per thread, with a
    ragged last round (P = 1,100,003).  With the depth prefix off every list is binned whole, so the sorted
    instances and the per-tile ranges must equal the oracle's element for element."""
    from dogs_amd.diff_gaussian_rasterization import _C
    n, W, H = 1_100_003, 256, 192
    s = small_scene(n, W, H, seed=41, sh_rest=3)
    s.scales = (s.scales * 0.5).contiguous()
    old = _C.set_prefix_per_tile(per_tile)
    try:
        col_o, radii_o, inv_o, st = oracle_forward(oracle, s, (0, 0, 0), deg=1)
        out = hip_forward(s, (0, 0, 0), hip_device, deg=1)
        assert out[0] == st.num_rendered
        np.testing.assert_array_equal(out[4].cpu().numpy(), radii_o)
        t_o, i_o, _ = st.sorted_list()
        t_h, i_h, e1 = hip_sorted_instances(out, W, H, hip_device, n)
        fT, nc, mc, rg = hip_image_state(out, W, H, hip_device)
        if per_tile:
            assert e1 == st.num_valid
            np.testing.assert_array_equal(t_h, t_o)
            np.testing.assert_array_equal(i_h, i_o)
            np.testing.assert_array_equal(rg, st.ranges())
        else:
            full = per_tile_lists(t_o, i_o, len(t_o))
            for t, lst in per_tile_lists(t_h, i_h, e1).items():
                assert lst == full[t][:len(lst)], f"tile {t}: not a prefix of the reference list"
        assert psnr(out[2].cpu().numpy(), col_o) > 80.0
    finally:
        _C.set_prefix_per_tile(old)


def test_cull_log_threshold_every_opacity(oracle, hip_device):
    """The binning's cull threshold logf(o / (1/255)) (rasterizer_impl.cu:151; gs_crlogf) equals the
    oracle's bit for bit on EVERY float opacity in (2^-24, 1] (2.0e8 values, in chunks of 2^25), so the (tile,
    Gaussian) keep decisions cannot differ at the threshold for any opacity."""
    from dogs_amd import _lib
    L = _lib.load()
    lo, hi = 0x33800001, 0x3F800001                 # (2^-24, 1]
    chunk = 1 << 25
    oracle.set_threads(0)
    checked = 0
    for start in range(lo, hi, chunk):
        bits = np.arange(start, min(start + chunk, hi), dtype=np.uint32)
        o = bits.view(np.float32)
        want = oracle.cull_log_threshold(o)
        od = torch.from_numpy(o).to(hip_device)
        got = torch.empty_like(od)
        _lib.check(L.dg_cull_log_threshold(od.numel(), od.data_ptr(), got.data_ptr(),
                                           _lib.stream_of(hip_device)))
        g = got.cpu().numpy()
        bad = np.flatnonzero(g.view(np.uint32) != want.view(np.uint32))
        assert bad.size == 0, [(float(o[i]).hex(), float(g[i]).hex(), float(want[i]).hex()) for i in bad[:8]]
        checked += o.size
    assert checked == hi - lo

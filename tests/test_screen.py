"""Split-precision variance screen (cdx_screen.hip) and the screened closure.

The closure estimates std² of every all-tip row with the bf16 screen and runs the exact fp64
whitened pass only for the fingertips that can still be their group's maximum (the variance cost
reads max_f log(100·std_f), optimize_pregrasp.py:733).  Parity bar: the screened closure equals the
unscreened fp64 closure (itself pinned to the reference fixtures by test_gpu_parity) to the rounding
of the refine pass's K-split (measured ≤ 1e-13 relative; asserted 1e-10), with identical NaN
positions and Kabsch masks, and no kept row's estimate outside the calibrated bound.
"""
import numpy as np
import pytest
import torch

from tests._helpers import rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"
OUTS = ("total_loss", "total_margin", "grad_q", "grad_comp", "grad_target", "grad_palm_pos", "grad_palm_ori")
TOL_EQ = 1e-10  # screened vs unscreened closure (same fp64 arithmetic, K-split rounding only)
# Along a 200-step trajectory the fingertips reach rows with var ≪ k0, where var = k0 − ‖V‖² cancels and
# the variance cost's ∇std/std amplifies the two passes' 1e-16 summation-order difference by ≈ k0/var
# (measured 1.3e-9 on g_q at the worst step, 1e-14 elsewhere): the per-step bar there is 1e-8.
TOL_TRAJ = 1e-8


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture(scope="module")
def banana2000():
    from compliancedex_amd.workloads import synthetic_banana_gpis
    return synthetic_banana_gpis(2000, device=DEV)


def _opt(hand="allegro"):
    from compliancedex_amd import ProbabilisticGraspOptimizer
    from compliancedex_amd.urdf import load_robot
    cfg = load_robot(hand)["config"]
    return cfg, ProbabilisticGraspOptimizer(hand, cfg["ee_link_name"], cfg["ee_link_offset"], ref_q=cfg["ref_q"],
                                            optimize_target=True, optimize_palm=True, device=DEV)


def _closure(opt, gpis, inputs, screen=True, delta_scale=1.0):
    q, comp, target, palm = inputs
    p = opt.problem(gpis, 1)
    delta = p.gpis.screen_delta
    if not screen:
        p.gpis.screen_delta = 0.0
    elif delta_scale != 1.0:  # debug margins (the closure's own descriptor copy): forces failed checks
        p.gpis.screen_delta = delta * delta_scale
    try:
        t = [torch.from_numpy(np.ascontiguousarray(a)).to(DEV).requires_grad_(True)
             for a in (q, comp, target, palm[:, :3], palm[:, 3:])]
        noise = torch.from_numpy(np.random.default_rng(7).random((3 * q.shape[0], 3, 3))).to(DEV)
        opt.closure(*t, 1, gpis, q.shape[0], kabsch_noise=noise)
        torch.cuda.synchronize()
        out = dict(total_loss=opt.total_loss.cpu().numpy(), total_margin=opt.total_margin.cpu().numpy(),
                   flip=opt.kabsch_flip.cpu().numpy())
        for k, x in zip(OUTS[2:], t):
            out[k] = x.grad.cpu().numpy()
        stats = opt.screen_stats(gpis, q.shape[0])
    finally:
        p.gpis.screen_delta = delta
    return out, stats


def _all_tip_queries(cfg, E, seed, center=None):
    from compliancedex_amd.workloads import prob_inputs
    from oracle.cdx_oracle import OracleChain, OracleProblem
    from compliancedex_amd.urdf import load_robot
    prob = OracleProblem(OracleChain(load_robot("allegro")["bodies"]), cfg["ee_link_name"], cfg["ee_link_offset"],
                         cfg["ref_q"], None)
    q, comp, target, palm = prob_inputs(cfg["ref_q"], E, seed=seed, spread=True, center=center)
    with torch.no_grad():
        pre = prob.forward_kinematics(torch.from_numpy(q), torch.from_numpy(palm)).double()
    tgt = torch.from_numpy(target)
    return (tgt + 0.8 * (pre - tgt)).reshape(-1, 3)


def test_screen_estimate_within_bound(banana2000):
    """The split-precision estimate of k0 − ‖L⁻¹k‖² against the fp64 pass on the bench's 16 384 all-tip rows:
    inside an eighth of the closure's margin Δ (= 32× the state's calibrated error; measured ≈ 3e-6·k0
    against a calibrated 2-4e-6·k0)."""
    from compliancedex_amd.gpis import exact_var
    cfg, _ = _opt()
    st = banana2000.native_state()
    X = _all_tip_queries(cfg, 4096, 1000).to(DEV)
    est = st.screen_var(X)
    ex = exact_var(st, X)
    err = float((est - ex).abs().max())
    k0 = float(banana2000.R) ** 3
    assert np.isfinite(est.cpu().numpy()).all()
    assert st.desc.screen_delta > 0
    assert err <= st.desc.screen_delta / 8, (err / k0, st.desc.screen_delta / k0)


def test_screen_var_c_abi_edges(banana2000):
    """M = 0 is a no-op; a null workspace / unprepared descriptor is rejected before any launch."""
    from compliancedex_amd import _native as N
    lib = N.load()
    st = banana2000.native_state()
    X = torch.zeros(4, 3, dtype=torch.float64, device=DEV)
    out = torch.zeros(4, dtype=torch.float64, device=DEV)
    assert lib.cdx_gpis_screen_var(st.desc, N.ptr(X), 0, N.ptr(out), None, None) == 0
    assert lib.cdx_gpis_screen_var(st.desc, N.ptr(X), 4, N.ptr(out), None, None) == -1
    bare = N.CdxGpis(X1=st.desc.X1, alpha=st.desc.alpha, Linv_t=st.desc.Linv_t, N=st.desc.N, N_pad=st.desc.N_pad)
    assert lib.cdx_gpis_screen_var(bare, N.ptr(X), 4, N.ptr(out), N.ptr(out), None) == -1


def test_screen_far_queries_are_nan(banana2000):
    """Beyond the safe radius (3.5R from the inducing points, where SA·Ã could leave fp16's range) the
    estimate is NaN, never a silently clamped number; near queries stay finite."""
    st = banana2000.native_state()
    X = torch.zeros(8, 3, dtype=torch.float64, device=DEV)
    X[:4] = banana2000.X1[:4].to(torch.float64)
    X[4:, 0] = torch.tensor([2.0, -3.0, 10.0, 1e6], dtype=torch.float64)
    est = st.screen_var(X).cpu().numpy()
    assert np.isfinite(est[:4]).all() and np.isnan(est[4:]).all(), est


def test_screened_closure_far_candidates(banana2000):
    """Candidates whose palm is 2 m away screen to NaN: their groups run the exact pass for every
    fingertip, and the closure still equals the unscreened one."""
    from compliancedex_amd.workloads import prob_inputs
    cfg, opt = _opt()
    q, comp, target, palm = prob_inputs(cfg["ref_q"], 2048, seed=99, spread=True)
    palm = palm.copy()
    palm[:128, 0] += 2.0
    a, st = _closure(opt, banana2000, (q, comp, target, palm), screen=True)
    b, _ = _closure(opt, banana2000, (q, comp, target, palm), screen=False)
    assert st["bound_misses"] == 0 and st["exact_rows"] >= 2048 + 3 * 128, st
    assert np.array_equal(a["flip"], b["flip"])
    for k in OUTS:
        assert rel_err(a[k], b[k]) <= TOL_EQ, (k, rel_err(a[k], b[k]))


@pytest.mark.parametrize("case", ["config2_E4096", "stored_banana_E1024", "config3_mug_E4096"])
def test_screened_closure_equals_fp64_closure(case, banana2000):
    """Screened vs unscreened closure on the same inputs: equal to TOL_EQ, NaNs and Kabsch masks
    identical; the exact pass ran for ≤ 1.25 fingertips per group and no kept estimate left its bound."""
    from compliancedex_amd.workloads import config3_gpis, prob_inputs, stored_gpis, surface_center
    cfg, opt = _opt()
    if case == "config2_E4096":
        gpis, E, center = banana2000, 4096, None
    elif case == "stored_banana_E1024":  # the smallest screened size (4096 all-tip rows), N = 361
        gpis, E, center = stored_gpis("banana", DEV), 1024, None
    else:
        _, gpis = config3_gpis(1, DEV)
        E, center = 4096, surface_center(gpis)
    inputs = prob_inputs(cfg["ref_q"], E, seed=321, spread=True, center=center)
    a, st = _closure(opt, gpis, inputs, screen=True)
    b, st0 = _closure(opt, gpis, inputs, screen=False)
    assert st0 is None and st is not None
    assert st["bound_misses"] == 0
    assert st["screened_rows"] == 4 * E
    assert E <= st["exact_rows"] <= 1.25 * E, st
    assert np.array_equal(a["flip"], b["flip"])
    for k in OUTS:
        assert rel_err(a[k], b[k]) <= TOL_EQ, (k, rel_err(a[k], b[k]))


@pytest.mark.parametrize("kernel", ["rbf", "joint"])
def test_screened_closure_other_gpis_kernels(kernel):
    """The screen's RBF (expm1 offset) and joint-kernel generation: the screened closure equals the
    unscreened one on an N = 2000 state fitted with that kernel (E = 1024, Leap hand for variety)."""
    from compliancedex_amd.gpis import GPIS
    from compliancedex_amd.workloads import prob_inputs, synthetic_banana_arrays
    X1, y, noise = synthetic_banana_arrays(2000)
    g = GPIS(0.08, 1.0, kernel=kernel)
    g.fit(torch.from_numpy(X1).to(DEV), torch.from_numpy(y).to(DEV), noise=torch.from_numpy(noise).to(DEV))
    g.bias = torch.tensor(1.0, dtype=torch.float64, device=DEV)
    cfg, opt = _opt("leap")
    inputs = prob_inputs(cfg["ref_q"], 1024, seed=11, spread=True)
    a, st = _closure(opt, g, inputs, screen=True)
    b, st0 = _closure(opt, g, inputs, screen=False)
    assert st0 is None and st is not None and st["bound_misses"] == 0
    assert 1024 <= st["exact_rows"] <= 4 * 1024
    assert np.array_equal(a["flip"], b["flip"])
    for k in OUTS:
        assert rel_err(a[k], b[k]) <= TOL_EQ, (k, rel_err(a[k], b[k]))


def test_small_closure_not_screened():
    """Below 4096 all-tip rows (config 1: E = 64) the closure runs the fp64 pass for every row: the
    screen's fixed cost would exceed what it saves (cdx_closure.hip SCREEN_MIN_ROWS)."""
    from compliancedex_amd.workloads import prob_inputs, stored_gpis
    cfg, opt = _opt()
    gpis = stored_gpis("banana", DEV)
    _, st = _closure(opt, gpis, prob_inputs(cfg["ref_q"], 64, seed=1, spread=True))
    assert st is None


def test_screened_closure_deterministic(banana2000):
    """Two screened closures on the same inputs and noise are bit-identical (the kept-row list is
    compacted in group order, not by atomics)."""
    from compliancedex_amd.workloads import prob_inputs
    cfg, opt = _opt()
    inputs = prob_inputs(cfg["ref_q"], 2048, seed=5, spread=True)
    a, _ = _closure(opt, banana2000, inputs)
    b, _ = _closure(opt, banana2000, inputs)
    for k in OUTS:
        assert np.array_equal(a[k], b[k], equal_nan=True), k


def _report(opt, gpis, E):
    r = opt.screen_report(gpis, E)
    assert r is not None
    return r


def test_screen_report_audits_discarded_rows(banana2000):
    """Every screened closure verifies itself (cdx_closure_screen_report): the exact pass also runs the
    discarded rows nearest the keep threshold — smallest normalised gap z = (lo − a_f)/Δ_f, the lowest
    1/8-octave z bins within CDX_SCREEN_AUDIT = 64 rows (≤ 4× that with the crossing bin) — and every
    kept and audited estimate is checked against its margin Δ_f.  On the bench workload: no miss, no
    audited row that turned out to be its group's maximum, no fault, no repair, the worst estimate error a
    small fraction of its margin, and every unaudited discarded row at least min_gap ≥ audit_cut > 1
    margins below its group's floor; the cumulative block counts the closures."""
    from compliancedex_amd.workloads import prob_inputs
    cfg, opt = _opt()
    inputs = prob_inputs(cfg["ref_q"], 4096, seed=1000, spread=True)
    _closure(opt, banana2000, inputs)
    r = _report(opt, banana2000, 4096)
    assert r["screened"] == 1 and r["screened_rows"] == 4 * 4096
    assert 0 < r["audited_rows"] <= 4 * 64 and r["audited_rows"] <= r["discarded_rows"], r
    assert r["exact_rows"] == 4 * 4096 - r["discarded_rows"] + r["audited_rows"], r
    assert r["bound_misses"] == r["audit_misses"] == r["audit_flips"] == r["faults"] == r["repaired"] == 0, r
    assert 0 < r["max_ratio"] < 0.5 and 0 < r["max_ratio_audit"] < 0.5, r
    assert r["min_gap"] >= r["audit_cut"] > 1.0, r  # the audit took the nearest rows
    n0 = r["cum_closures"]
    _closure(opt, banana2000, inputs)
    r2 = _report(opt, banana2000, 4096)
    assert r2["cum_closures"] == n0 + 1
    assert r2["cum_audited_rows"] >= r["audited_rows"] + r2["audited_rows"] or n0 == 0
    # reset zeroes the cumulative block only
    from compliancedex_amd import _native as N
    p = opt.problem(banana2000, 1)
    N.check(N.load().cdx_closure_screen_reset(p, 4096, N.ptr(opt._last_ws), N.stream_ptr(opt._last_ws.device)), "reset")
    r3 = _report(opt, banana2000, 4096)
    assert r3["cum_closures"] == 0 and r3["cum_audited_rows"] == 0 and r3["audited_rows"] == r2["audited_rows"]


def test_screened_closure_adversarial_far_queries(banana2000):
    """The regime the margin's row scale max(1, ‖Ṽ‖²/k0) has to cover: palms pushed 5 cm … 3.5R away
    along random directions (log-uniform), so the fingertip queries spread from the surface to beyond
    the screen's safe radius (NaN estimates → whole group exact).  Screened = unscreened to TOL_EQ;
    no margin miss, audit miss or fault; some far groups really were screened."""
    from compliancedex_amd.workloads import prob_inputs
    cfg, opt = _opt()
    E = 4096
    q, comp, target, palm = prob_inputs(cfg["ref_q"], E, seed=4242, spread=True)
    rng = np.random.default_rng(4242)
    R = float(banana2000.R)
    d = np.exp(rng.uniform(np.log(0.05), np.log(3.5 * R), E))
    u = rng.standard_normal((E, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    palm = palm.copy()
    palm[:, :3] += d[:, None] * u
    a, st = _closure(opt, banana2000, (q, comp, target, palm), screen=True)
    r = _report(opt, banana2000, E)
    b, _ = _closure(opt, banana2000, (q, comp, target, palm), screen=False)
    assert r["bound_misses"] == r["audit_misses"] == r["audit_flips"] == r["faults"] == 0, r
    # far groups are screened too: fewer exact rows than "every group beyond 5 cm runs all four"
    assert E <= r["exact_rows"] < 3 * E, r
    assert np.array_equal(a["flip"], b["flip"])
    for k in OUTS:
        assert rel_err(a[k], b[k]) <= TOL_EQ, (k, rel_err(a[k], b[k]))


def test_optimize_trajectory_screened_equals_unscreened_every_step(banana2000):
    """A 200-iteration config-2 optimise loop (fused Adam, best iterate, clamps), screened: at EVERY
    step the closure's loss, margins and five gradients equal the unscreened fp64 closure's on the
    same parameters and Kabsch noise to TOL_TRAJ (NaN candidates identical), and the loop's
    cumulative screen record shows no
    miss, fault or audit flip (so no closure repaired itself).
    (Two separately run trajectories are not compared: the screened and unscreened exact passes sum
    V in different K-splits — 1e-16 relative — and 200 Adam steps amplify that to 1e-9 by step 26.)"""
    from compliancedex_amd import ProbabilisticGraspOptimizer
    from compliancedex_amd.workloads import prob_inputs
    cfg, opt = _opt()
    opt.num_iters = 200
    E = 4096
    q, comp, target, palm = prob_inputs(cfg["ref_q"], E, seed=77, spread=True)
    opt.palm_offset = torch.from_numpy(palm).to(DEV)
    args = [torch.from_numpy(np.ascontiguousarray(x)).to(DEV) for x in (q, target, comp)]
    ref = ProbabilisticGraspOptimizer("allegro", cfg["ee_link_name"], cfg["ee_link_offset"], ref_q=cfg["ref_q"],
                                      optimize_target=True, optimize_palm=True, device=DEV)
    p_ref = ref.problem(banana2000, 1)
    assert p_ref.gpis.screen_delta > 0
    p_ref.gpis.screen_delta = 0.0  # this optimiser's own descriptor copy: the full fp64 pass

    class Tape:  # per-step Kabsch noise, drawn on the device from a seeded generator
        def __init__(self):
            self.g = torch.Generator(device=DEV).manual_seed(2024)

        def __getitem__(self, s):
            return torch.rand(3 * E, 3, 3, generator=self.g, device=DEV, dtype=torch.float64)

    keys = ("total_loss", "total_margin", "g_q", "g_comp", "g_target", "g_palm_pos", "g_palm_ori")
    worst = torch.zeros(len(keys), dtype=torch.float64, device=DEV)
    steps = []

    def hook(s, out, st):
        o2 = ref._outputs(E, 4, 16, 3, torch.device(DEV))
        ref._closure_into(p_ref, st["q"], st["comp"], st["target"], st["pp"], st["po"], st["noise"], o2, seed=0)
        for i, k in enumerate(keys):
            a, b = out[k], o2[k]
            fin = torch.isfinite(b)
            assert torch.equal(torch.isfinite(a), fin), (s, k)  # NaN candidates where the reference has them
            e = torch.where(fin, (a - b).abs(), 0).max() / torch.where(fin, b.abs(), 0).max().clamp(min=1e-300)
            worst[i] = torch.maximum(worst[i], e)
        steps.append(s)

    opt.optimize(*args, 1, banana2000, verbose=False, noise_tape=Tape(), step_hook=hook)
    rep = opt.last_screen_report
    assert steps == list(range(200)) and opt.screen_repairs == 0
    assert rep["cum_closures"] == 200 and rep["cum_bound_misses"] == rep["cum_faults"] == rep["cum_repairs"] == 0, rep
    assert rep["cum_audit_misses"] == rep["cum_audit_flips"] == 0 and rep["cum_audited_rows"] > 200 * 16, rep
    w = worst.cpu().numpy()
    assert (w <= TOL_TRAJ).all(), dict(zip(keys, w))


def test_screened_graph_replay_matches_eager(banana2000):
    """hipGraph capture of the screened closure (E = 1024: 4096 all-tip rows, the screen's threshold):
    the captured fork/join of the side-stream GPIS mean, the device-side refine row count and the
    audit replay bit-identically to the eager loop; screen_report reads the graph's own workspace."""
    from compliancedex_amd.workloads import prob_inputs
    cfg, opt = _opt()
    opt.num_iters = 12
    E = 1024
    q, comp, target, palm = prob_inputs(cfg["ref_q"], E, seed=31, spread=True)
    opt.palm_offset = torch.from_numpy(palm).to(DEV)
    args = [torch.from_numpy(np.ascontiguousarray(x)).to(DEV) for x in (q, target, comp)]
    opt._seed = 9
    eager = [r.cpu().numpy() for r in opt.optimize(*args, 1, banana2000, verbose=False)]
    rep_e = opt.last_screen_report
    opt._seed = 9
    graph = [r.cpu().numpy() for r in opt.optimize(*args, 1, banana2000, verbose=False, graph=True)]
    rep_g = opt.last_screen_report
    opt._seed = 9
    replay = [r.cpu().numpy() for r in opt.optimize(*args, 1, banana2000, verbose=False, graph=True)]
    assert rep_e is not None and rep_g is not None
    assert rep_g["cum_closures"] == 12 and rep_g["exact_rows"] == rep_e["exact_rows"], (rep_e, rep_g)
    for x, y, z in zip(eager, graph, replay):
        assert np.array_equal(x, y, equal_nan=True) and np.array_equal(x, z, equal_nan=True)


_FIRST_CAPTURE = r"""
import sys, numpy as np, torch
sys.path.insert(0, {repo!r})
from compliancedex_amd import ProbabilisticGraspOptimizer
from compliancedex_amd.urdf import load_robot
from compliancedex_amd.workloads import prob_inputs, stored_gpis
cfg = load_robot("allegro")["config"]
g = stored_gpis("banana", "cuda")
q, comp, target, palm = prob_inputs(cfg["ref_q"], 1024, seed=3, spread=True)
res = []
for graph in (True, False):  # the capture is this process's FIRST screened closure
    opt = ProbabilisticGraspOptimizer("allegro", cfg["ee_link_name"], cfg["ee_link_offset"], palm_offset=palm,
                                      ref_q=cfg["ref_q"], optimize_target=True, optimize_palm=True, device="cuda",
                                      num_iters=6, seed=5)
    a = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (q, target, comp)]
    res.append([r.cpu().numpy() for r in opt.optimize(*a, 1, g, verbose=False, graph=graph)])
    assert opt.last_screen_report is not None and opt.last_screen_report["cum_faults"] == 0
for x, y in zip(*res):
    assert np.array_equal(x, y, equal_nan=True)
print("first-capture ok")
"""


def test_screened_graph_first_capture_creates_side_stream():
    """The per-device side stream is created lazily by the first screened closure — here inside a
    hipGraph capture, in a fresh process (one child, bounded by a timeout): the capture and replay
    still equal the eager loop bit for bit."""
    import subprocess
    import sys
    from tests.conftest import REPO
    r = subprocess.run([sys.executable, "-c", _FIRST_CAPTURE.format(repo=REPO)], capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and "first-capture ok" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])


_KABSCH_CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, {repo!r})
from compliancedex_amd import ProbabilisticGraspOptimizer
from compliancedex_amd.urdf import load_robot
from compliancedex_amd.workloads import prob_inputs, synthetic_banana_gpis
cfg = load_robot("allegro")["config"]
g = synthetic_banana_gpis(2000, device="cuda")
q, comp, target, palm = prob_inputs(cfg["ref_q"], 4096, seed=321, spread=True)
out = {{}}
for mode in ("given", "device"):
    opt = ProbabilisticGraspOptimizer("allegro", cfg["ee_link_name"], cfg["ee_link_offset"], palm_offset=palm,
                                      ref_q=cfg["ref_q"], optimize_target=True, optimize_palm=True, device="cuda",
                                      seed=77)
    t = [torch.from_numpy(np.ascontiguousarray(a)).cuda().requires_grad_(True)
         for a in (q, comp, target, palm[:, :3], palm[:, 3:])]
    noise = (torch.from_numpy(np.random.default_rng(7).random((3 * 4096, 3, 3))).cuda() if mode == "given" else None)
    opt.closure(*t, 1, g, 4096, kabsch_noise=noise)
    torch.cuda.synchronize()
    out[mode + "_loss"] = opt.total_loss.cpu().numpy()
    out[mode + "_margin"] = opt.total_margin.cpu().numpy()
    out[mode + "_flip"] = opt.kabsch_flip.cpu().numpy()
    for i, x in enumerate(t):
        out[mode + "_g%d" % i] = x.grad.cpu().numpy()
np.savez({path!r}, **out)
print("kabsch child ok")
"""


def test_kabsch_records_ahead_bit_identical(tmp_path):
    """The screened closure computes the Kabsch records (SVD of the weighted cross-covariance) on a
    side stream ahead of the level kernel (closure_kabsch_kernel, ahead of the mean on its stream); with
    CDX_KABSCH_AHEAD=0 the level kernel runs the SVD itself.  Both give bit-identical losses, margins, Kabsch masks and gradients, with
    the Kabsch noise given and drawn on the device.  (The switch is read once per process: one child
    per setting.)"""
    import os
    import subprocess
    import sys
    from tests.conftest import REPO
    res = {}
    for ahead in ("1", "0"):
        path = str(tmp_path / f"k{ahead}.npz")
        env = dict(os.environ, CDX_KABSCH_AHEAD=ahead)
        r = subprocess.run([sys.executable, "-c", _KABSCH_CHILD.format(repo=REPO, path=path)], capture_output=True,
                           text=True, timeout=240, env=env)
        assert r.returncode == 0 and "kabsch child ok" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])
        res[ahead] = np.load(path)
    a = res["0"]
    for mode in ("1",):
        b = res[mode]
        assert set(a.files) == set(b.files)
        for k in a.files:
            assert np.array_equal(a[k], b[k], equal_nan=True), (mode, k)
    assert np.isfinite(a["given_loss"]).sum() > 4000


_VARLATE_CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, {repo!r})
from compliancedex_amd import ProbabilisticGraspOptimizer
from compliancedex_amd.urdf import load_robot
from compliancedex_amd.workloads import prob_inputs, synthetic_banana_gpis
cfg = load_robot("allegro")["config"]
g = synthetic_banana_gpis(2000, device="cuda")
out = {{}}
for E in (4096, 256):  # screened (side-stream level kernel) and unscreened (below the screen's row threshold)
    q, comp, target, palm = prob_inputs(cfg["ref_q"], E, seed=321, spread=True)
    opt = ProbabilisticGraspOptimizer("allegro", cfg["ee_link_name"], cfg["ee_link_offset"], palm_offset=palm,
                                      ref_q=cfg["ref_q"], optimize_target=True, optimize_palm=True, device="cuda",
                                      seed=77)
    t = [torch.from_numpy(np.ascontiguousarray(a)).cuda().requires_grad_(True)
         for a in (q, comp, target, palm[:, :3], palm[:, 3:])]
    opt.closure(*t, 1, g, E)
    torch.cuda.synchronize()
    out["e%d_loss" % E] = opt.total_loss.cpu().numpy()
    out["e%d_margin" % E] = opt.total_margin.cpu().numpy()
    out["e%d_flip" % E] = opt.kabsch_flip.cpu().numpy()
    for i, x in enumerate(t):
        out["e%d_g%d" % (E, i)] = x.grad.cpu().numpy()
np.savez({path!r}, **out)
print("varlate child ok")
"""


def test_variance_cost_in_combine_matches_level_kernel(tmp_path):
    """CDX_VAR_LATE (default 1): the level kernel leaves the variance cost uncertainty·max_f log(100·std_f)
    (optimize_pregrasp.py:733) out and the combine kernel adds it — loss term and, through the all-tip
    interpolation, its ∇std gradient — so that the level kernel can run beside the std passes.  Against
    CDX_VAR_LATE=0 (the level kernel adds it, round-2 arithmetic): losses, margins and Kabsch masks
    bit-identical (the variance term is the last operand of the level loss's left-to-right sum); the tip
    and target gradients differ only by the order of one addition (c·(a + b) vs c·a + c·b): 1e-13 of the
    largest entry.  Screened E = 4096 (level kernel on the side stream) and unscreened E = 256."""
    import os
    import subprocess
    import sys
    from tests.conftest import REPO
    res = {}
    for vl in ("1", "0"):
        path = str(tmp_path / f"v{vl}.npz")
        env = dict(os.environ, CDX_VAR_LATE=vl)
        r = subprocess.run([sys.executable, "-c", _VARLATE_CHILD.format(repo=REPO, path=path)], capture_output=True,
                           text=True, timeout=240, env=env)
        assert r.returncode == 0 and "varlate child ok" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])
        res[vl] = np.load(path)
    a, b = res["0"], res["1"]
    assert set(a.files) == set(b.files)
    for k in a.files:
        if k.endswith(("_loss", "_margin", "_flip")):
            assert np.array_equal(a[k], b[k], equal_nan=True), k
        else:
            fin = np.isfinite(a[k])
            assert np.array_equal(fin, np.isfinite(b[k])), k
            scale = max(np.abs(a[k][fin]).max(), 1e-300)
            assert np.abs(a[k][fin] - b[k][fin]).max() <= 1e-13 * scale, (k, np.abs(a[k][fin] - b[k][fin]).max() / scale)
    assert np.isfinite(a["e4096_loss"]).sum() > 3000


def test_injected_error_joins_side_stream(banana2000):
    """Every error return after the screened closure has forked its side stream (Kabsch records, mean,
    level kernel) joins it first (cdx_closure.hip: joined()).  cdx_debug_fail_next_closure makes the next
    closure fail at one of three points — after the screen / selection / fork, after the exact pass,
    after the ∇std pass — through the failed-launch error path.  Eagerly: the call raises, the stream
    drains, and the next closure gives the unfailed results bit for bit.  Under hipGraph capture: the
    call raises and the capture still ends cleanly (an unjoined fork would make capture_end fail with
    its own error instead of the closure's)."""
    from compliancedex_amd import _native as N
    from compliancedex_amd.workloads import prob_inputs
    cfg, opt = _opt()
    E = 1024  # 4096 all-tip rows: screened, side stream forked
    q, comp, target, palm = prob_inputs(cfg["ref_q"], E, seed=41, spread=True)
    opt.palm_offset = torch.from_numpy(palm).to(DEV)
    t = [torch.from_numpy(np.ascontiguousarray(x)).to(DEV) for x in (q, comp, target, palm[:, :3], palm[:, 3:])]
    noise = torch.from_numpy(np.random.default_rng(5).random((3 * E, 3, 3))).to(DEV)
    lib = N.load()

    def run():
        opt.closure(*t, 1, banana2000, E, kabsch_noise=noise)
        return [x.detach().cpu().numpy().copy() for x in (opt.total_loss, opt.total_margin, opt.kabsch_flip)]

    ref = run()
    torch.cuda.synchronize()
    for stage in (1, 2, 3):
        N.check(lib.cdx_debug_fail_next_closure(stage), "cdx_debug_fail_next_closure")
        with pytest.raises(RuntimeError, match="cdx_closure failed"):
            opt.closure(*t, 1, banana2000, E, kabsch_noise=noise)
        torch.cuda.synchronize()
        for a, b in zip(run(), ref):
            assert np.array_equal(a, b, equal_nan=True), stage
        N.check(lib.cdx_debug_fail_next_closure(stage), "cdx_debug_fail_next_closure")
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with pytest.raises(RuntimeError, match="cdx_closure failed"):
            with torch.cuda.stream(side):
                with torch.cuda.graph(g, stream=side):
                    opt.closure(*t, 1, banana2000, E, kabsch_noise=noise)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        del g
        for a, b in zip(run(), ref):
            assert np.array_equal(a, b, equal_nan=True), stage
    N.check(lib.cdx_debug_fail_next_closure(0), "cdx_debug_fail_next_closure")



@pytest.mark.parametrize("scale", [1e-3, 1e-9])
def test_failed_checks_repair_the_closure(scale, banana2000):
    """Injected screen misses: the closure's margins shrunk to scale × Δ (1e-3: kept and audited rows
    miss it; 1e-9: groups keep only their leader and the true maximum is often discarded).  Every check
    that fails makes the same closure repair itself — every all-tip row through the exact pass, the
    unscreened selection — so the reference-API closure() returns the unscreened fp64 closure's loss,
    margins, Kabsch masks and five gradients (TOL_EQ), and the report says it repaired."""
    from compliancedex_amd.workloads import prob_inputs
    cfg, opt = _opt()
    E = 4096
    inputs = prob_inputs(cfg["ref_q"], E, seed=1000, spread=True)
    a, _ = _closure(opt, banana2000, inputs, screen=True, delta_scale=scale)
    r = _report(opt, banana2000, E)
    b, _ = _closure(opt, banana2000, inputs, screen=False)
    assert r["repaired"] == 1 and r["cum_repairs"] >= 1, r
    assert r["bound_misses"] + r["audit_misses"] + r["audit_flips"] + r["faults"] > 0, r
    assert np.array_equal(a["flip"], b["flip"])
    for k in OUTS:
        assert rel_err(a[k], b[k]) <= TOL_EQ, (k, rel_err(a[k], b[k]))
    c, _ = _closure(opt, banana2000, inputs, screen=True)  # the calibrated margins again: no repair
    r2 = _report(opt, banana2000, E)
    assert r2["repaired"] == 0, r2
    for k in OUTS:
        assert rel_err(c[k], b[k]) <= TOL_EQ, (k, rel_err(c[k], b[k]))


_ENV_REPAIR_CHILD = r"""
import sys, json, numpy as np
sys.path.insert(0, {repo!r})
from tests.test_screen import _closure, _opt, _report, OUTS
from compliancedex_amd.workloads import prob_inputs, synthetic_banana_gpis
from tests._helpers import rel_err
g = synthetic_banana_gpis(2000, device="cuda")
cfg, opt = _opt()
E = 4096
inputs = prob_inputs(cfg["ref_q"], E, seed=1000, spread=True)
a, st = _closure(opt, g, inputs, screen=True, delta_scale=1e-3)
r = _report(opt, g, E)
b, _ = _closure(opt, g, inputs, screen=False)
err = max(rel_err(a[k], b[k]) for k in OUTS)
print(json.dumps(dict(repaired=r["repaired"], audited=r["audited_rows"], exact=r["exact_rows"], err=err,
                      flips_equal=bool(np.array_equal(a["flip"], b["flip"])))))
"""


def test_env_switches_cannot_disable_the_repair():
    """with CDX_SCREEN_REPAIR=0, CDX_SCREEN_AUDIT=0 and CDX_NO_SCREEN=1 in the environment, the shipped
    library still screens, audits the discarded rows and repairs a closure whose checks fail (margins 1e-3 × Δ), so it
    returns the unscreened fp64 closure's results (TOL_EQ).  (Read once per process: a child process.)"""
    import json
    import os
    import subprocess
    import sys
    from tests.conftest import REPO
    env = dict(os.environ, CDX_SCREEN_REPAIR="0", CDX_SCREEN_AUDIT="0", CDX_NO_SCREEN="1")
    r = subprocess.run([sys.executable, "-c", _ENV_REPAIR_CHILD.format(repo=REPO)], capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["repaired"] == 1 and res["audited"] > 0 and 0 < res["exact"] < 4 * 4096, res
    assert res["flips_equal"] and res["err"] <= TOL_EQ, res


@pytest.mark.parametrize("fused", [True, False])
def test_optimize_with_failed_checks_equals_unscreened(fused, banana2000):
    """A 30-iteration optimise loop with injected misses (margins 1e-3 × Δ), through the fused loop and
    the reference loop (fused=False, torch.optim.Adam): every closure repairs itself on the device (no
    host sync per step), cum_repairs = 30, and at every step (fused) / at the end (both) the results
    equal the unscreened loop's on the same noise to the K-split rounding (per step TOL_EQ; the final
    best iterate 1e-8 after 30 Adam steps)."""
    from compliancedex_amd import ProbabilisticGraspOptimizer
    from compliancedex_amd.workloads import prob_inputs
    cfg, opt = _opt()
    opt.num_iters = 30
    E = 4096
    q, comp, target, palm = prob_inputs(cfg["ref_q"], E, seed=78, spread=True)
    args = [torch.from_numpy(np.ascontiguousarray(x)).to(DEV) for x in (q, target, comp)]

    def run(o, delta_scale, hook=None):
        o.palm_offset = torch.from_numpy(palm).to(DEV)
        p = o.problem(banana2000, 1)
        d0 = p.gpis.screen_delta
        p.gpis.screen_delta = d0 * delta_scale
        g = torch.Generator(device=DEV).manual_seed(99)
        tape = [torch.rand(3 * E, 3, 3, generator=g, device=DEV, dtype=torch.float64) for _ in range(30)]
        try:
            res = o.optimize(*[x.clone() for x in args], 1, banana2000, verbose=False, noise_tape=tape, fused=fused,
                             step_hook=hook)
        finally:
            p.gpis.screen_delta = d0
        return [x.detach().cpu().numpy() for x in res]

    ref = ProbabilisticGraspOptimizer("allegro", cfg["ee_link_name"], cfg["ee_link_offset"], ref_q=cfg["ref_q"],
                                      optimize_target=True, optimize_palm=True, device=DEV)
    ref.num_iters = 30
    p_ref = ref.problem(banana2000, 1)
    keys = ("total_loss", "total_margin", "g_q", "g_comp", "g_target", "g_palm_pos", "g_palm_ori")
    worst = [0.0]

    def hook(s, out, st):
        d0 = p_ref.gpis.screen_delta
        p_ref.gpis.screen_delta = 0.0
        o2 = ref._outputs(E, 4, 16, 3, torch.device(DEV))
        ref._closure_into(p_ref, st["q"], st["comp"], st["target"], st["pp"], st["po"], st["noise"], o2, seed=0)
        p_ref.gpis.screen_delta = d0
        for k in keys:
            x, y = out[k], o2[k]
            fin = torch.isfinite(y)
            assert torch.equal(torch.isfinite(x), fin), (s, k)
            e = float(torch.where(fin, (x - y).abs(), 0).max() / torch.where(fin, y.abs(), 0).max().clamp(min=1e-300))
            worst[0] = max(worst[0], e)

    got = run(opt, 1e-3, hook if fused else None)
    rep = opt.last_screen_report
    assert rep["cum_closures"] == 30 and rep["cum_repairs"] == 30, rep
    assert worst[0] <= TOL_EQ, worst
    want = run(ref, 0.0)
    for x, y in zip(got, want):
        fin = np.isfinite(y)
        assert np.array_equal(np.isfinite(x), fin)
        assert np.abs(x[fin] - y[fin]).max() <= 1e-8 * max(np.abs(y[fin]).max(), 1e-300)

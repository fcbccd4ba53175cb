"""The fp32 convolution plan table (conv32.hip kTuned, queried through the
host-side planner -- no GPU needed) and the MFL_C32_PLANS override used by
whole-step plan sweeps (scripts/gpu_plans/r4_plans*.txt)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = """
from metisfl_amd.ops._native import ops
o = ops(); o.set_conv32_mode(1)
for s in [(32,16,16,128,128,3,3,1,1), (32,32,32,64,64,3,3,1,1), (32,4,4,512,512,3,3,1,1)]:
    d, w = o.conv32_plan(1, *s), o.conv32_plan(2, *s)
    print(d[0], d[1], d[2], w[0], w[1], w[2])
"""


def _plans(env_extra=None):
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("MFL_C32_PLANS", None)
    env.update(env_extra or {})
    out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, cwd=ROOT,
                         timeout=300)
    assert out.returncode == 0, out.stderr
    return [tuple(int(v) for v in line.split()) for line in out.stdout.strip().splitlines()]


def test_paired_backward_plans_fill_one_wave():
    """Every stride-1 3x3 backward pair of ResNet-18 at batch 32 runs 64x64
    tiles (the pairing condition); the 16x16x128 pair is dgrad 2 x wgrad 7
    slices = 764 workgroups, one wave of 3 per CU (profiles/r4/plans/)."""
    l2, l1, l4 = _plans()
    assert l2 == (64, 64, 2, 64, 64, 7)
    assert l1[:2] == (64, 64) and l1[3:5] == (64, 64)
    assert l4[:2] == (64, 64) and l4[3:5] == (64, 64)
    tiles_d = (32 * 16 * 16 // 64) * (128 // 64)
    tiles_w = (128 // 64) * (128 * 9 // 64)
    assert tiles_d * l2[2] + tiles_w * l2[5] <= 3 * 256
    # 4x4x512: dgrad 4 x wgrad 1 = 832 workgroups, one wave of 4 per CU on the
    # co-located learners' 2-stage pair ring (profiles/r4/ns/tq_*.log)
    assert l4[2] == 4 and l4[5] == 1
    assert (32 * 4 * 4 // 64) * (512 // 64) * l4[2] + (512 // 64) * (512 * 9 // 64) * l4[5] <= 4 * 256


def test_plan_override_env():
    l2, l1, _ = _plans({"MFL_C32_PLANS": "1,16,128,128,3,1,4;2,16,128,128,3,1,3"})
    assert l2[2] == 4 and l2[5] == 3
    assert l1 == _plans()[1]  # other shapes untouched


def test_infeasible_split_override_snaps_to_a_feasible_count():
    """1,024 k-tiles cannot split into 56 equal shares: the request runs 54
    slices of 19 tiles (it used to leave the plan without a tile, and the
    weight gradient unwritten)."""
    _, l1, _ = _plans({"MFL_C32_PLANS": "2,32,64,64,3,1,56"})
    assert l1[5] == 54


def test_regime_overrides_stay_feasible_at_other_batch_sizes():
    """The co-located regime's plan overrides are batch independent (set
    process-wide before the learners' graphs are captured).  At batch 512 -- the
    evaluation twin of a learner built after the regime was set -- the 2-way
    8x8x256 dgrad split would have 2,048 tiles, past the in-launch split-K
    reduce's counter block: the planner must fall back to a feasible plan
    instead of raising (the GPU suite hit this in test_eval_twin_gpu.py once a
    two-learner test had set the regime)."""
    code = """
from metisfl_amd.models.colocated import CoLocatedLearners
from metisfl_amd.ops._native import ops
o = ops(); o.set_conv32_mode(1)
o.set_conv32_plan_overrides(CoLocatedLearners.plans)
for s in [(512,8,8,256,256,3,3,1,1), (512,16,16,128,128,3,3,1,1), (32,8,8,256,256,3,3,1,1)]:
    d = o.conv32_plan(1, *s)
    print(d[0], d[1], d[2])
"""
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("MFL_C32_PLANS", None)
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, cwd=ROOT,
                         timeout=300)
    assert out.returncode == 0, out.stderr
    p512, p512b, p32 = [tuple(int(v) for v in l.split()) for l in out.stdout.strip().splitlines()]
    assert p512[2] >= 1 and p512b[2] >= 1
    tiles = (512 * 8 * 8 // p512[0]) * (256 // p512[1])
    assert p512[2] == 1 or tiles <= 1024
    assert p32 == (64, 64, 2)  # the override itself still applies at batch 32

"""bench.py's contract pieces that need no GPU: the N-rank launcher (gloo
dry run through torch.distributed.run, 127.0.0.1), the world-size check, the
algorithmic FLOP model and the stamped PMC lookup."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=timeout, cwd=REPO)


@pytest.mark.timeout(300)
def test_gpus_flag_launches_that_many_ranks():
    r = _run(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout                    # rank 0 only
    assert json.loads(lines[0]) == {"dry_run": True, "n_gpus": 2}


def test_world_size_must_match_gpus_flag():
    r = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "1"})
    assert r.returncode != 0 and "--gpus 2" in r.stderr


def test_algorithmic_flops_are_three_forwards():
    import bench
    t, b = 64, 1
    total = sum(bench.algorithmic_flops(k, b, t) for k in
                ("k_pw_fa", "k_conv_fa", "k_pw_fb", "k_conv_fb", "k_pw_ba", "k_conv_ba",
                 "k_pw_bb", "k_conv_bb", "k_wgrad"))
    fwd = t * (2 * bench.conv_flops() + 6 * bench.gate_flops())
    # backward: dgrad of both convs (frame 0's conv^T(w_inh) is dead) + wgrads,
    # 1x1 dgrad + wgrad (frame 0's attention backward is dead)
    assert total == 3 * fwd - bench.conv_flops() - 4 * bench.gate_flops()
    assert abs(3 * fwd / 1e9 - 41.9) < 0.1               # SURVEY §8(d) 41.91 GFLOP/clip


def test_pmc_traffic_needs_matching_library_stamp(tmp_path, monkeypatch):
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "r99_pmc_traffic.json").write_text(json.dumps(
        {"note": "B=256 T=64 bf16", "lib_version": "pt_cell x src abc",
         "kernels": {"k_pw_bb": {"traffic_bytes": 123}}}))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    assert bench.pmc_traffic("k_pw_bb", 256, 64, "bf16", "pt_cell x src abc") == 123
    assert bench.pmc_traffic("k_pw_bb", 256, 64, "bf16", "pt_cell x src def") is None
    assert bench.pmc_traffic("k_pw_bb", 128, 64, "bf16", "pt_cell x src abc") is None


def test_roofline_follows_survey_8d():
    """bench.py reports the dominant kernel against the roofline SURVEY.md §8(d)
    binds it to (MFMA for every kernel with a k x k conv), the step's §8(d)
    FLOPs (41.91 GFLOP per 64-frame clip) and the PMC step bytes against
    §8(d)'s 17.2 MB-per-clip minimum; the r04 numbers reproduce from the
    committed profiles (0.173 of MFMA for k_fused_fa, 66.1 GB/step)."""
    import bench
    assert abs(bench.step_flops_8d(1, 64) - 41.91e9) < 0.01e9
    r, fl, by, avg = bench.kernel_roofline("k_fused_fa", 65.86e-3 * 640, 640, 256, 64, 10, "bf16", 4, True)
    assert r["bound"] == "mfma" and fl == 256 * (bench.conv_flops() + 4 * bench.gate_flops())
    assert abs(r["frac"] - 0.1728) < 1e-3 and r["frac"] == r["mfma_frac"]
    r, *_ = bench.kernel_roofline("k_pw_ba", 57e-3 * 640, 640, 256, 64, 10, "bf16", 4, True)
    assert r["bound"] == "hbm"
    sb = bench.pmc_step_bytes(256, 64, "bf16", "pt_cell 0.2 gfx950 src 0fc1382ba8c5")
    assert sb is not None and abs(sb / 1e9 - 66.15) < 0.1
    assert abs(sb / (256 * 64 * bench.BYTES_8D_FRAME) - 15.0) < 0.1
    assert bench.pmc_step_bytes(256, 64, "bf16", "some other library") is None

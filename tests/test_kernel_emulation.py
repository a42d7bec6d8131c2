"""CPU emulation of the Check interpreter's step boundary (no GPU).

tools/cpuemu builds the kernel SOURCES for the host, one lane per wavefront.  Built with
KETO_GUARD=1, every lane runs exactly one transition per load slot, so every pseudo
transition crosses a step boundary -- the path a lane takes on the GPU when its 24-transition
budget runs out.  The GPU parity suite (golden fixtures + random worlds) must still agree with
the oracle.  Without the S_FSCAN rule in check.hip's transition loop 41 of those cases failed.
The frontier engine's tests (test_gpu_frontier.py) run in the same emulation: one-lane waves
and blocks, so its wave-level scans and block allocation take their degenerate paths.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
def test_one_transition_per_step_matches_oracle(tmp_path):
    lib = tmp_path / "libketo_emu_g1.so"
    jobs = str(min(8, os.cpu_count() or 1))
    subprocess.run(["make", "-s", "-j", jobs, "-C", os.path.join(ROOT, "tools", "cpuemu"),
                    f"OBJDIR={tmp_path / 'obj'}", f"LIB={lib}", "OPT=-O1 -DKETO_GUARD=1"],
                   check=True, timeout=600)
    env = dict(os.environ, KETO_MI355X_ALLOW_OVERRIDE="tools", KETO_MI355X_LIB_OVERRIDE=str(lib))
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "gpu", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_gpu_parity.py"), os.path.join(ROOT, "tests", "test_gpu_frontier.py"),
                        os.path.join(ROOT, "tests", "test_gpu_reach.py"),
                        "-k", "golden or random_worlds or synthetic_small or frontier or routed or reach"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert " passed" in r.stdout


@pytest.mark.slow
def test_one_transition_per_step_is_address_clean(tmp_path):
    """The same worst-case schedule under AddressSanitizer, with the DFS interpreter answering
    every batch (KETO_FRONTIER=0): no out-of-range access from any interpreter state at a step
    boundary.  (the round-1 waterfall-dispatch fault.)"""
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not asan or not os.path.isabs(asan):
        pytest.skip("no libasan")
    lib = tmp_path / "libketo_emu_asan.so"
    jobs = str(min(8, os.cpu_count() or 1))
    subprocess.run(["make", "-s", "-j", jobs, "-C", os.path.join(ROOT, "tools", "cpuemu"),
                    f"OBJDIR={tmp_path / 'obj'}", f"LIB={lib}",
                    "OPT=-O1 -fsanitize=address -fno-omit-frame-pointer -DKETO_GUARD=1"],
                   check=True, timeout=900)
    env = dict(os.environ, KETO_MI355X_ALLOW_OVERRIDE="tools", KETO_MI355X_LIB_OVERRIDE=str(lib), KETO_FRONTIER="0",
               LD_PRELOAD=asan, ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-m", "gpu", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_gpu_parity.py"), "-k", "golden or random_worlds or synthetic_small"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=1200)
    assert "AddressSanitizer" not in r.stdout + r.stderr, (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


@pytest.mark.slow
def test_unserved_lanes_lose_operands_but_stay_in_range(tmp_path):
    """The round-1 waterfall variant's failure mode: lanes that sit out a step
    after their operands were loaded (-DKETO_EMU_SKIP=3: every third lane-step on average) run
    their next transition on cleared operands.  That gives wrong decisions -- the invariant the
    shipped kernel keeps -- but never an out-of-range access under AddressSanitizer."""
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not asan or not os.path.isabs(asan):
        pytest.skip("no libasan")
    lib = tmp_path / "libketo_emu_skip.so"
    jobs = str(min(8, os.cpu_count() or 1))
    subprocess.run(["make", "-s", "-j", jobs, "-C", os.path.join(ROOT, "tools", "cpuemu"),
                    f"OBJDIR={tmp_path / 'obj'}", f"LIB={lib}",
                    "OPT=-O1 -fsanitize=address -fno-omit-frame-pointer -DKETO_EMU_SKIP=3"],
                   check=True, timeout=900)
    env = dict(os.environ, KETO_MI355X_ALLOW_OVERRIDE="tools", KETO_MI355X_LIB_OVERRIDE=str(lib), KETO_FRONTIER="0",
               LD_PRELOAD=asan, ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-m", "gpu", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_gpu_parity.py"), "-k", "golden or random_worlds"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=1200)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out, out[-3000:]
    assert " failed" in r.stdout, "lost operands should change decisions (else the knob did nothing)"


@pytest.mark.slow
def test_patched_snapshots_exact_under_emulation(tmp_path):
    """keto_store_snapshot_patch and _advance under the CPU emulation (one lane at a time, so even
    routed queries' goal counts are deterministic): patched and advanced snapshots equal full builds
    in every answer, goal count and Expand tree; the store's content index through churn and a mass
    delete (tests/test_gpu_store.py, the patch, advance and index cases)"""
    lib = tmp_path / "libketo_emu_patch.so"
    jobs = str(min(8, os.cpu_count() or 1))
    subprocess.run(["make", "-s", "-j", jobs, "-C", os.path.join(ROOT, "tools", "cpuemu"),
                    f"OBJDIR={tmp_path / 'obj'}", f"LIB={lib}", "OPT=-O1"], check=True, timeout=600)
    env = dict(os.environ, KETO_MI355X_ALLOW_OVERRIDE="tools", KETO_MI355X_LIB_OVERRIDE=str(lib))
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "gpu", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_gpu_store.py"), "-k", "patch or advance or index"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "12 passed" in r.stdout

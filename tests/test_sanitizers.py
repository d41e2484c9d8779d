"""Host AddressSanitizer + UBSan build of the C++ CPU simulator.  GPU sanitizers are not
available on the MI355X pool, so the device kernels are covered by numerics tests instead."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPU = os.path.join(ROOT, "quantum_distributed_machine_learning_ris_channel_estimation_amd", "csrc", "cpu")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_cpu_simulator_asan_ubsan(tmp_path):
    exe = tmp_path / "qsim_cpu_check"
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-fopenmp", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           "-fno-sanitize-recover=undefined", os.path.join(CPU, "qsim_cpu.cpp"),
           os.path.join(CPU, "tests", "qsim_cpu_check.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0", OMP_NUM_THREADS="2")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout

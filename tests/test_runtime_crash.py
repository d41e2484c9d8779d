"""The native crash report (csrc/hip/runtime.hip qd_install_crash_handler, installed by _native.hip_lib): a host
fault in native code prints the native frames (library + offset), then still reaches Python's faulthandler and the
default action (exit by the signal).  Runs on the CPU: loading the HIP library needs no GPU."""
import os
import subprocess
import sys
import textwrap

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "quantum_distributed_machine_learning_ris_channel_estimation_amd", "lib", "libqdml_hip.so")


@pytest.mark.skipif(not os.path.exists(LIB), reason="libqdml_hip.so not built")
def test_native_segfault_reports_native_and_python_frames():
    script = textwrap.dedent(f"""
        import faulthandler, sys
        faulthandler.enable()
        sys.path.insert(0, {REPO!r})
        from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
        lib = nat.hip_lib(build_if_missing=False)
        def replay_like_frame():
            lib.qd_crash_for_test()
        replay_like_frame()
        print("unreachable", flush=True)
    """)
    p = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=240)
    assert p.returncode == -11, (p.returncode, p.stderr[-3000:])
    err = p.stderr
    assert "[qdml] SIGSEGV @0x0000000000000000" in err, err[-3000:]
    assert "native frames" in err and "libqdml_hip.so" in err, err[-3000:]   # (the faulting library is named)
    assert "replay_like_frame" in err, err[-3000:]                           # (faulthandler still ran after it)
    assert "unreachable" not in p.stdout


@pytest.mark.skipif(not os.path.exists(LIB), reason="libqdml_hip.so not built")
def test_crash_handler_can_be_turned_off():
    script = textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {REPO!r})
        from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
        nat.hip_lib(build_if_missing=False).qd_crash_for_test()
    """)
    p = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, QDML_CRASH_HANDLER="0"))
    assert p.returncode == -11 and "[qdml] SIGSEGV" not in p.stderr


@pytest.mark.skipif(not os.path.exists(LIB), reason="libqdml_hip.so not built")
def test_crash_report_also_goes_to_the_crash_log(tmp_path):
    """QDML_CRASH_LOG: the native frames also land in a file (pytest's capture of fd 2 dies with the process)."""
    log = tmp_path / "crash.log"
    script = textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {REPO!r})
        from quantum_distributed_machine_learning_ris_channel_estimation_amd import _native as nat
        nat.hip_lib(build_if_missing=False).qd_crash_for_test()
    """)
    p = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, QDML_CRASH_LOG=str(log)))
    assert p.returncode == -11
    text = log.read_text()
    assert "[qdml] SIGSEGV" in text and "libqdml_hip.so" in text and "end of native frames" in text, text

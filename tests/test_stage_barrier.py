"""StageBarrier, the barrier of the devices= threads (fs_internal.h), under
the interleaving of ADVICE r3: the thread that completes a stage goes on and
fails the next one before a slow waiter of the completed stage wakes.  The
waiter must still see its stage as passed (the stage's verdict is fixed when
the last thread arrives); before the fix it saw the later failure, skipped
its remaining barriers and left its peers waiting.  Native driver:
tests/native/stage_barrier_check.cpp (2000 rounds)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_stage_verdict_survives_a_later_failure(tmp_path):
    exe = str(tmp_path / "stage_barrier_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread",
                    os.path.join(HERE, "native", "stage_barrier_check.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr

"""Zero-copy host rings (ingot_gpu_host_map): the cases live in
tests/hostmap_cases.py and run here in ONE child pytest process, so the
page-locking and unmapping of host memory they do (hipHostRegister /
hipHostUnregister of pageable buffers) never shares a process with the rest
of the GPU suite.  Needs an MI355X: `pytest -m gpu`."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.gpu
def test_host_map_cases_in_a_child_process():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, "-u", "-m", "pytest", "tests/hostmap_cases.py", "-x", "-q",
           "-p", "no:cacheprovider", "--timeout", "90", "--timeout-method", "thread"]
    try:
        p = subprocess.run(cmd, cwd=ROOT, env=dict(os.environ), capture_output=True, text=True,
                           timeout=110)
    except subprocess.TimeoutExpired as e:
        pytest.fail(f"hostmap cases timed out:\n{e.stdout}\n{e.stderr}")
    print(p.stdout[-4000:])
    assert p.returncode == 0, p.stdout[-6000:] + p.stderr[-3000:]
    assert " passed" in p.stdout and "skipped" not in p.stdout, p.stdout[-2000:]

"""Planner accuracy on the device: the modelled one-GPU step -- layer costs
timed on this GPU at two batch sizes (per-call fixed cost + per-sample slope), one chain timing
of the whole spine to calibrate their sum, the fused optimizer pass -- against the measured step
of the same model, batch and optimizer through ``madnn.distribute``: within +-20 %."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench"))


@pytest.mark.parametrize("model,batch", [("resnet50", 512), ("gpt2-medium", 16)])
def test_modelled_step_within_20_percent(cuda, model, batch, tmp_path):
    """Planned and measured in a fresh process, as a job would: inside the long-lived test process
    (hundreds of earlier GPU tests, their allocator pools and tuned-choice caches) the measured
    GPT-2 step ran 40 % slower than the same case alone, which is no statement about the planner."""
    import json
    import subprocess

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "plan.json"
    subprocess.run([sys.executable, os.path.join(repo, "bench", "plan_accuracy.py"), "--cases", f"{model}:{batch}",
                    "--json-out", str(out)], check=True, timeout=300, cwd=repo)
    r = json.load(open(out))[0]
    assert r["measured_costs"]
    assert 0.8 <= r["ratio"] <= 1.2, r

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
def test_modelled_step_within_20_percent(cuda, model, batch):
    from plan_accuracy import run_case

    r = run_case(model, batch, steps=5, warmup=3)
    assert r["measured_costs"]
    assert 0.8 <= r["ratio"] <= 1.2, r

"""Every ``examples/*.py`` runs end to end at world size 2 on CPU (gloo) through the launcher,
at tiny sizes.  The CIFAR example is the reference's only validation artifact
(/root/reference/cifar_example/sgd-torchad_nn-cifar.lua:260-301: a confusion matrix, the test
accuracy and a results file): it must learn (> 50 % on the 10-class synthetic set) and write
``SgdAuto--Size:<n>--Batch:<b>.txt``."""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow

CASES = {
    "cifar_auto_dp.py": ["-size", "1200", "-iterations", "3", "-learningRate", "0.01", "-batchSize", "10"],
    "mp_mlp.py": [],
    "gpt2_pipeline.py": ["--model", "gpt2-tiny", "--stages", "2", "--microbatches", "2", "--batch", "4", "--seq", "32",
                         "--steps", "2"],
    "llama_hybrid.py": ["--model", "llama3-tiny", "--batch", "4", "--seq", "32", "--steps", "2"],
    "bert_ckpt_adam.py": ["--model", "bert-tiny", "--batch", "4", "--seq", "32", "--steps", "2"],
}


def test_every_example_is_covered():
    have = sorted(f for f in os.listdir(os.path.join(ROOT, "examples")) if f.endswith(".py"))
    assert have == sorted(CASES)


@pytest.mark.parametrize("script", sorted(CASES))
def test_example_runs_at_world_2(script, tmp_path):
    env = dict(os.environ, MADNN_LOG_LEVEL="WARNING", OMP_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    cmd = [sys.executable, "-m", "madnn.launch", "--nproc", "2", "--timeout", "400",
           os.path.join(ROOT, "examples", script), *CASES[script]]
    res = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=480)
    out = res.stdout + res.stderr
    assert res.returncode == 0, out[-4000:]
    if script == "cifar_auto_dp.py":
        acc = float(re.search(r"accuracy ([0-9.]+)%", out).group(1))
        assert acc > 50.0, out[-2000:]
        files = [f for f in os.listdir(tmp_path) if f.startswith("SgdAuto--Size:1200--Batch:10")]
        assert files, os.listdir(tmp_path)
        text = open(os.path.join(tmp_path, files[0])).read()
        assert "Accuracy:" in text and "World size: 2" in text
    elif script in ("gpt2_pipeline.py", "llama_hybrid.py", "bert_ckpt_adam.py"):
        assert re.search(r"step 1 loss [0-9.]+", out), out[-2000:]
    else:
        assert "iter 15 loss" in out, out[-2000:]

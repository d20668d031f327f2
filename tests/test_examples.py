"""The S7 examples run end to end (CPU)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples"))


def test_environment_example(tmp_path):
    import environment_example
    out = tmp_path / "lt.gif"
    assert environment_example.main(["--steps", "8", "--oracle", "push", "--out", str(out)]) == 0
    assert out.exists() and out.stat().st_size > 0


def test_dataset_example():
    import dataset_example
    assert dataset_example.main(["--episodes", "2", "--window", "3", "--batch", "2"]) == 0

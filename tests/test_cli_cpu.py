"""rtrec_amd.train_movielens keeps the reference CLI (scripts/train_movielens.py:41-49)
and refuses to run without a ROCm device (no CPU training path)."""
import pytest


def test_reference_arguments_and_defaults():
    from rtrec_amd import train_movielens as tm
    a = tm.build_parser().parse_args([])
    assert (a.data_path, a.epochs, a.batch_size, a.lr, a.embedding_dim, a.device, a.num_negatives) == \
        ("ml-1m", 50, 1024, 0.001, 128, "auto", 16)
    a = tm.build_parser().parse_args(["--epochs", "1", "--batch-size", "256", "--embedding-dim", "64"])
    assert (a.epochs, a.batch_size, a.embedding_dim, a.dropout) == (1, 256, 64, 0.2)


def test_no_cpu_path():
    import torch
    from rtrec_amd import train_movielens as tm
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="no CPU training path"):
        tm.run(tm.build_parser().parse_args(["--synthetic", "--epochs", "1"]))

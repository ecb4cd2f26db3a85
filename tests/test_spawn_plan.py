"""The GPU test harness's device assignment (tests/spawn_ranks.py), checked without a GPU."""
import pytest

from spawn_ranks import device_plan, rank_device


def test_shared_plan_is_the_default():
    plan, env = device_plan(4, 8)
    assert plan == "shared"
    assert env["MP4X_DEVICE_BACKEND"] == "gloo" and env["MP4X_DEVICE_INDEX"] == "0"
    assert [rank_device(plan, r) for r in range(4)] == [0, 0, 0, 0]
    assert "GPU_MAX_HW_QUEUES" not in env                      # 4 ranks x 4 queues fit
    assert device_plan(8, 1)[1]["GPU_MAX_HW_QUEUES"] == "2"     # 8 ranks share the queue slots


@pytest.mark.parametrize("p,ndev,plan", [(2, 8, "multi"), (8, 8, "multi"), (8, 4, "shared"), (2, 1, "shared"),
                                         (4, 0, "shared")])
def test_auto_plan(p, ndev, plan):
    got, env = device_plan(p, ndev, "auto")
    assert got == plan
    if plan == "multi":
        assert env["MP4X_DEVICE_BACKEND"] == "nccl" and "MP4X_DEVICE_INDEX" not in env
        assert [rank_device(got, r) for r in range(p)] == list(range(p))
    else:
        assert env["MP4X_DEVICE_BACKEND"] == "gloo"


def test_multi_plan_needs_enough_gpus():
    with pytest.raises(ValueError):
        device_plan(4, 2, "multi")
    with pytest.raises(ValueError):
        device_plan(2, 2, "bogus")


def test_multi_dryrun_plans_shared(monkeypatch):
    """MP4X_TEST_MULTI_DRYRUN=1 (VERDICT r5 Next #2): the cross-GPU tests run on one GPU with gloo
    instead of skipping; without the knob the multi plan still needs a GPU per rank."""
    monkeypatch.setenv("MP4X_TEST_MULTI_DRYRUN", "1")
    plan, env = device_plan(8, 1, "multi")
    assert plan == "shared" and env["MP4X_DEVICE_BACKEND"] == "gloo" and env["GPU_MAX_HW_QUEUES"] == "2"
    monkeypatch.setenv("MP4X_TEST_MULTI_DRYRUN", "0")
    with pytest.raises(ValueError):
        device_plan(8, 1, "multi")

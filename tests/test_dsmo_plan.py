"""Host-side plan of the distributed SMO (csrc/hip/dsmo.hip: dsmo_shape + check_plan): for every size
and team count the teams must cover every point, fit one sweep, and -- for the one-launch
rehearsal -- be co-resident on one GPU.  Runs on the CPU (the device library loads without a GPU)."""
import pytest

from svm355.parallel.dsmo import plan


@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize("n", [2, 100, 3000, 6000, 20000, 60000, 120000, 250000, 500000, 1000000])
@pytest.mark.parametrize("one_launch", [False, True])
def test_plan_covers_every_point_within_the_sweep(n, world, one_launch):
    try:
        p = plan(n, world, 256, one_launch)
    except Exception:
        # only a one-launch rehearsal of a very large n may have no shape (too many workgroups for one GPU)
        assert one_launch and n >= 500000
        return
    total = p["workgroups_per_team"] * world
    assert p["slice"] == p["threads"] * p["points_per_thread"]
    assert p["team_width"] == p["workgroups_per_team"] * p["slice"]
    assert total * p["slice"] >= n
    assert total <= 64 * p["records_per_lane"] <= 256
    assert (total if one_launch else p["workgroups_per_team"]) <= 256


def test_headline_plans():
    # 60k over 8 GPUs: 8 workgroups x 256 threads x 4 points per GPU, one 64-record sweep
    assert plan(60000, 8) == {"threads": 256, "points_per_thread": 4, "workgroups_per_team": 8,
                              "records_per_lane": 1, "slice": 1024, "team_width": 8192}
    p = plan(60000, 1)
    assert p["workgroups_per_team"] * p["slice"] >= 60000 and p["records_per_lane"] == 1

"""Extract the reference's embedded known-answer vectors into tests/golden/*.json.

Runs only in the build container (reads /root/reference, which the GPU box does not
have).  It copies DATA only — the numeric arrays the reference's plotting scripts
embed as outputs of earlier runs — never code:
  * utils/hybrid_astar/plot.py:47-51  path of utils/hybrid_astar/test_hybrid_astar.cpp
  * utils/dubins_paths.py:6           Dubins<double> RSL path, start (0,0,0) goal (20,-20,pi/2)
  * utils/vehicle_mode.py:12          VehicleModel<double>::simulate_action positions
The scenario inputs (parameters, obstacles, start/goal) are transcribed from the
harness sources cited in each fixture's "source" field.
"""
import json
import math
import re
from pathlib import Path

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parents[1] / "tests" / "golden"


def grab_array(path, name):
    text = (REF / path).read_text()
    m = re.search(name + r"\s*=\s*np\.array\((\[.*?\])\)", text, re.S)
    if not m:
        raise SystemExit(f"no array {name} in {path}")
    body = m.group(1)
    if not re.fullmatch(r"[\s\d\.\-\+eE,\[\]]+", body):
        raise SystemExit("unexpected characters in array literal")
    return json.loads(body)


def main():
    OUT.mkdir(parents=True, exist_ok=True)
    steering_deg = [-30.0, -15.0, 0.0, 15.0, 30.0]
    harness = {
        "source": "utils/hybrid_astar/test_hybrid_astar.cpp:13-98 (inputs), utils/hybrid_astar/plot.py:47-51 (path, printed with %g)",
        "params": {
            "dubins_shot_interval": 300, "dubins_shot_interval_decay": 10,
            "grid_resolution": 0.5, "obstacle_threshold": 0.75, "obstacle_prob_min": 0.1,
            "obstacle_prob_max": 0.95, "obstacle_prob_free": 0.4, "grid_size": 60,
            "grid_2d_allow_diag_moves": 1, "step_size": 0.75, "max_lat_acc": 4.0,
            "max_long_dec": 2.0, "wheelbase": 2.269, "rear_to_cg": 1.1,
            "apf_rep_constant": 1.0, "apf_active_angle_expr": "float(M_PI/4)",
            "num_angle_bins": 72, "num_actions": 1,
            "steering_deg": steering_deg, "steering_expr": "float(angle_f * M_PI / 180.0f)",
            "curvature_weights": [0, 0, 0, 0, 0],
        },
        "lines": [[21.9, 4.5, 21.9, 31.5], [20.4, 33.0, 38.4, 33.0], [10.5, 4.5, 10.5, 40.5], [9.0, 42.0, 39.0, 42.0]],
        "line_conf": 0.6, "line_width": 1.25,
        "boxes": [[18.0, 22.8, 3.5, 2.9], [14.25, 28.5, 2.0, 5.3], [18.0, 34.8, 3.5, 2.9]],
        "box_conf": 0.75, "apf_added_radius": 2.5, "cycles": 5,
        "start": [18.0, 18.0, "M_PI_2"], "goal": [26.0, 36.0, 0.0], "vel": 2.0,
        "path_start_to_goal": grab_array("utils/hybrid_astar/plot.py", "path"),
    }
    (OUT / "harness_60.json").write_text(json.dumps(harness, indent=1))
    dub = {
        "source": "utils/vehicle_dubins/test_vehicle_dubins.cpp:17-44 (inputs), utils/dubins_paths.py:6 (path)",
        "step_size": 0.5, "wheelbase": 2.269, "rear_to_cg": 1.1, "max_steering_deg": 30.0,
        "start": [0.0, 0.0, 0.0], "goal": [20.0, -20.0, "M_PI_2"],
        "path": grab_array("utils/dubins_paths.py", "path"),
    }
    (OUT / "dubins_rsl.json").write_text(json.dumps(dub, indent=1))
    veh = {
        "source": "utils/vehicle_dubins/test_vehicle_dubins.cpp:17-24,61-67 (inputs), utils/vehicle_mode.py:12 (positions)",
        "step_size": 0.5, "max_lat_acc": 4.0, "wheelbase": 2.269, "rear_to_cg": 1.1, "num_angle_bins": 72,
        "num_actions": 1, "steering_deg": [-30.0, -20.0, -10.0, 0.0, 10.0, 20.0, 30.0],
        "vmin_sqr0": 16.0, "curvature_index0": 3,
        "actions": [6, 6, 6, 6, 6, 6, 5, 5, 5, 5, 4, 4, 4, 4, 4, 3, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 4, 4, 4, 4],
        "positions": grab_array("utils/vehicle_mode.py", "path"),
    }
    (OUT / "vehicle_chain.json").write_text(json.dumps(veh, indent=1))
    print("wrote", sorted(p.name for p in OUT.glob("*.json")))


if __name__ == "__main__":
    main()

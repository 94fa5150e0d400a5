"""Writes tests/golden/reference_kat.json: the RNG-free known-answer tests
that the reference's own test-suite asserts, transcribed as data (inputs,
expected outputs, tolerances) with their source lines. These pin the CPU
oracle to the reference (the reference itself is Rust and cannot be built or
run in this environment: no cargo/rustc, no vendored crates).

Run: python tools/make_reference_kat.py
"""
import json
import math
import os

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "tests", "golden", "reference_kat.json")

kat = {
    "build_tree": {
        "source": "src/nuts.rs:521-586 (test_build_tree)",
        "target": {"kind": "DiffableGaussian2D", "mean": [0.0, 1.0], "cov": [[4.0, 2.0], [2.0, 3.0]]},
        "inputs": {"q": [0.0, 1.0], "p": [2.0, 3.0], "g": [4.0, 5.0], "logu": -2.0, "v": -1,
                   "j": 3, "eps": 0.01, "joint0": 0.1},
        "expected": {
            "qm": [-0.1584001, 0.76208336], "pm": [1.9800036, 2.9718253],
            "gm": [-7.91236e-5, 7.9358295e-2],
            "qp": [-0.0198, 0.97025], "pp": [1.98, 2.9749503], "gp": [-1.250e-05, 9.925e-03],
            "qprime": [-0.0198, 0.97025], "gprime": [-1.250e-05, 9.925e-03],
            "n": 0, "s": True, "n_alpha": 8, "logp_prime": -2.8777454, "alpha": 0.0006866617,
        },
        "tol": {"vec_rel": 1e-5, "vec_abs": 1e-6, "logp_abs": 1e-6, "alpha_abs": 1e-8},
    },
    "find_reasonable_epsilon": {
        "source": "src/nuts.rs:508-519 (test_find_reasonable_epsilon)",
        "target": {"kind": "StandardNormal"},
        "inputs": {"q": [0.0, 1.0], "p": [1.0, 0.0]},
        "expected": 2.0,
    },
    "chain_1": {
        "source": "src/nuts.rs:588-601 (test_chain_1)",
        "target": {"kind": "DiffableGaussian2D", "mean": [0.0, 1.0], "cov": [[4.0, 2.0], [2.0, 3.0]]},
        "inputs": {"init": [0.0, 1.0], "n_collect": 1, "n_discard": 0, "target_accept": 0.8},
        "expected": [[0.0, 1.0]],
        "tol": {"rel": 1e-5, "abs": 1e-6},
    },
    "mct_rhat": {
        "source": "src/stats.rs:734-783 (test_rhat_f32_1, test_rhat_f64_1, test_rhat_f64_2)",
        "tol": 10 * 1.1920929e-07,
        "cases": [
            {"steps": [[[0.0, 1.0, 0.0, 1.0], [1.0, 2.0, 0.0, 2.0], [0.0, 0.0, 0.0, 2.0]],
                       [[1.0, 2.0, 2.0, 0.0], [1.0, 1.0, 1.0, 1.0], [0.0, 1.0, 0.0, 0.0]]],
             "expected": [math.sqrt(2.0), 1.0801234, 0.8944273, 0.8660254]},
            {"steps": [[[0.0, 1.0, 0.0, 1.0], [1.0, 2.0, 0.0, 2.0], [0.0, 0.0, 0.0, 2.0]],
                       [[1.0, 2.0, 2.0, 0.0], [1.0, 1.0, 1.0, 1.0], [0.0, 1.0, 0.0, 0.0]]],
             "expected": [math.sqrt(2.0), 1.0801234, 0.8944271, 0.8660254]},
            {"steps": [[[1.0, 0.0, 0.0, 1.0], [1.0, 0.0, 0.0, 1.0], [0.0, 1.0, 0.0, 2.0]],
                       [[1.0, 2.0, 0.0, 2.0], [1.0, 2.0, 0.0, 0.0], [2.0, 0.0, 1.0, 2.0]]],
             "expected": [1.0 / math.sqrt(2.0), 0.74535599, 1.0, 1.5]},
        ],
    },
    "autocov": {
        "source": "src/stats.rs:808-839 (test_single_param, test_two_params_1)",
        "tol": 1e-6,
        "cases": [
            {"x": [[1.0], [2.0], [3.0], [4.0]], "expected": [[1.25], [0.3125], [-0.375], [-0.5625]]},
            {"x": [[1.0, 0.3], [2.0, 2.0], [3.0, -2.0], [4.0, 5.0]],
             "expected": [[1.25, 6.516875], [0.3125, -3.7889063], [-0.375, 1.4721875],
                          [-0.5625, -0.94171875]]},
        ],
    },
    "iso_gauss": {
        "source": "src/distributions.rs:580-614 (iso_gauss_unnorm_logp_test_1..3)",
        "note": "p = exp(unnorm_logp(x) - d/2 (ln 2 + ln pi + 2 ln std))",
        "cases": [
            {"std": 1.0, "x": [1.0], "expected_p": 0.24197072451914337, "tol": 1e-7},
            {"std": 2.0, "x": [0.42, 9.6], "expected_p": 3.864661987252467e-7, "tol": 1e-15},
            {"std": 3.0, "x": [1.0, 2.0, 3.0], "expected_p": 0.001080393185560214, "tol": 1e-8},
        ],
    },
    "gaussian2d_logp": {
        "source": "src/distributions.rs:820-839 (test_gaussian2d_logp)",
        "mean": [0.0, 0.0], "cov": [[1.0, 0.0], [0.0, 1.0]], "x": [0.5, -0.5],
        "expected": -2.0878770664093453, "tol": 1e-10,
    },
    "mass_matrix": {
        "source": "src/generic_nuts.rs:1427-1440 (diagonal_mass_matrix_kinetic_and_inv_mul_are_consistent)",
        "var": [4.0, 9.0], "p": [2.0, 3.0], "expected_kinetic": 1.0,
        "expected_inv_mul": [0.5, 1.0 / 3.0], "tol": 1e-12,
    },
    "ess_iid_uniform": {
        "source": "src/stats.rs:841-865 (ess_1): 4 chains x 1000 iid U(0,1), one parameter",
        "expected": {"ess_min_gt": 3800.0, "rhat_max_lt": 1.01},
    },
}

os.makedirs(os.path.dirname(OUT), exist_ok=True)
with open(OUT, "w") as f:
    json.dump(kat, f, indent=1)
print("wrote", OUT)

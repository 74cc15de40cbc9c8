"""libfst_amd.optimize_bench: the reference bench CLI's options, inputs and JSON schema
(bench/optimize-bench.zig:104-158, :160-199, :505-541); GPU runs check avg_states against
the oracle's result sizes for the same scenario."""
import json

import pytest

import oracle_ffi as O
from libfst_amd import optimize_bench as B


def test_inputs_match_the_reference_acceptors():
    # buildRepeatedLabelAcceptor / buildLinearAcceptorWithAlphabet: label = byte + 1
    assert [b + 1 for b in B.input_bytes("repeat", 5, 12)] == [1] * 5
    assert [b + 1 for b in B.input_bytes("branch", 7, 3)] == [1, 2, 3, 1, 2, 3, 1]
    assert [b + 1 for b in B.input_bytes("linear", 300, 3)][254:257] == [255, 1, 2]


def test_defaults_and_rejects():
    a = B.parse_args([])
    assert (a.len, a.transducer_len, a.branches, a.iters, a.warmup, a.format) == \
        (4096, 0, 3, 80, 5, "text")
    assert B.parse_args(["--branches", "0"]).branches == 1
    with pytest.raises(SystemExit):
        B.parse_args(["--iters", "0"])
    assert B.main(["--scenario", "optimize_transducer"]) == 2


def oracle_states(scenario, L, T, Bn):
    kind, gen, op = B.PLAN[scenario]
    lhs = O.compile_string(B.input_bytes(kind, L, Bn))
    if op == "sp":
        rc, r = O.shortest_path(lhs, 1)
        return r.num_states
    name = {0: "ambiguous", 1: "eps_dense", 2: "branching_frozen_src"}[gen]
    blob = O.freeze(O.gen(name, T, Bn))
    if op == "compose":
        rc, r = O.compose(lhs, blob)
    elif op == "lazy":
        rc, r = O.compose_shortest_path(lhs, blob, 1)
    else:
        rc, lat = O.compose(lhs, blob)
        rc, r = O.shortest_path(lat, 1)
    assert rc == O.OR_OK
    return r.num_states


@pytest.mark.gpu
@pytest.mark.parametrize("scenario", sorted(B.PLAN))
def test_scenarios_json(scenario, capsys):
    L, T, Bn = 12, 32, 5
    assert B.main(["--scenario", scenario, "--len", str(L), "--transducer-len", str(T),
                   "--branches", str(Bn), "--iters", "2", "--warmup", "1",
                   "--format", "json", "--per-iter", "true"]) == 0
    lines = [json.loads(x) for x in capsys.readouterr().out.strip().splitlines()]
    assert [x["iter"] for x in lines[:2]] == [0, 1]
    rec = lines[-1]
    assert set(rec) == {"scenario", "len", "transducer_len", "branches", "warmup", "iters",
                        "total_ns", "avg_ns", "min_ns", "max_ns", "avg_states"}
    assert rec["avg_states"] == oracle_states(scenario, L, T, Bn)


@pytest.mark.gpu
def test_batch_flag(capsys):
    assert B.main(["--scenario", "compose_frozen_lazy_shortest_path_ambiguous", "--len", "64",
                   "--transducer-len", "4096", "--branches", "12", "--iters", "2",
                   "--warmup", "1", "--format", "json", "--batch", "4096"]) == 0
    rec = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert rec["batch"] == 4096 and rec["avg_states"] == 65 and rec["strings_per_s"] > 0

"""libfst_amd: MI355X-native (gfx950) batched frozen-FST compose + 1-best engine.

Drop-in for ontypehq/libfst's fst_compose_frozen_shortest_path / fst_compose_frozen
hot path; see include/fst.h, include/fst_batch.h and DESIGN.md.
"""
from .fst import (  # noqa: F401
    BENCH_AMBIGUOUS, BENCH_BRANCHING, BENCH_EPS_DENSE, FST_EPSILON, FST_INVALID_HANDLE,
    FST_NO_STATE, FST_PATH_CYCLE, FST_PATH_EMPTY, FST_PATH_ERROR_N, FST_PATH_OK,
    FST_PATH_OUTPUT_FULL, FST_PATH_OVERFLOW, FST_PATH_UNSUPPORTED, FST_SEM_EAGER, FST_SEM_LAZY,
    Fst, MutableFst, compose_frozen, compose_frozen_shortest_path,
    coalescer_state, compose_frozen_shortest_path_batch, last_launch_stats, lib, pipeline_batch,
    shortest_path)

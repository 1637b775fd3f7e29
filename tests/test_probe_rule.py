"""CPU: when check_sets asks the device to skip its candidate-0 probe launch
(gpu_check._long_hint_miss -> PF_FLAG_NO_PROBE, pathfeas.hip check_enqueue): only for a long
program with variables whose host hint model leaves a root false."""
from types import SimpleNamespace

from mythril_amd import ir
from mythril_amd.smt import gpu_check


def _prog(n_vars, n_ins, n_roots, n_sat):
    info = [0] * 17
    info[0], info[6], info[10], info[13] = n_vars, n_ins, n_roots, n_sat
    return SimpleNamespace(native_result=SimpleNamespace(info=info))


def test_long_hint_miss():
    miss = gpu_check._long_hint_miss
    assert miss(_prog(101, 1846, 8, 7), 400)          # q18's bucket of the sample
    assert not miss(_prog(101, 1846, 8, 8), 400)      # the hint holds: probe pays
    assert not miss(_prog(3, 60, 5, 4), 400)          # short: the probe walk is cheap
    assert not miss(_prog(0, 900, 2, 0), 400)         # no variables: candidate 0 is all of them
    assert not miss(_prog(101, 1846, 8, 7), 0)        # probe split off: rule off
    assert not miss(SimpleNamespace(), 400)           # not a native program


def test_flag_value_matches_header():
    import os
    import re

    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "include", "pf_bytecode.h")).read()
    assert int(re.search(r"#define PF_FLAG_NO_PROBE (\d+)u", src).group(1)) == ir.FLAG_NO_PROBE

"""The library's hardware-queue bookkeeping (csrc/orbpl_runtime.cpp): it
records the queue count the HIP runtime really uses, changes
GPU_MAX_HW_QUEUES only when it is unset or ORBPL_HW_QUEUES asks, never when
the runtime was already started, and the LSD split decision follows the
recorded count, not the environment. Each case loads liborbpl.so in a fresh
process (the constructor runs at load time); no HIP call is made."""
import json
import os
import subprocess
import sys

import pytest

from _pkg import PKG_DIR

PROBE = r"""
import ctypes as C, json, os, sys
L = C.CDLL(sys.argv[1])
q, st, sb, sp = C.c_int(), C.c_int(), C.c_int(), C.c_int()
assert L.orbpl_hw_queue_state(C.byref(q), C.byref(st), C.byref(sb), C.byref(sp)) == 0
libc = C.CDLL(None)
libc.getenv.restype = C.c_char_p
v = libc.getenv(b"GPU_MAX_HW_QUEUES")   # the C environment (os.environ is a start-up copy)
print(json.dumps(dict(queues=q.value, started=st.value, set_by_lib=sb.value, split=sp.value,
                      env=v.decode() if v else None)))
"""


def _state(**env):
    e = {k: v for k, v in os.environ.items()
         if k not in ("GPU_MAX_HW_QUEUES", "ORBPL_HW_QUEUES", "ORBPL_ASSUME_RUNTIME_STARTED",
                      "ORBPL_LSD_SPLIT")}
    e.update(env)
    r = subprocess.run([sys.executable, "-c", PROBE, str(PKG_DIR / "liborbpl.so")], env=e,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("env,want", [
    # unset: filled in with 16, split on
    ({}, dict(queues=16, started=0, set_by_lib=1, split=1, env="16")),
    # the user's (the GPU box's) 4 is left alone, split off
    ({"GPU_MAX_HW_QUEUES": "4"}, dict(queues=4, started=0, set_by_lib=0, split=0, env="4")),
    ({"GPU_MAX_HW_QUEUES": "12"}, dict(queues=12, started=0, set_by_lib=0, split=1, env="12")),
    # an explicit request wins over the user's value before the runtime starts
    ({"GPU_MAX_HW_QUEUES": "4", "ORBPL_HW_QUEUES": "16"},
     dict(queues=16, started=0, set_by_lib=1, split=1, env="16")),
    ({"ORBPL_HW_QUEUES": "0"}, dict(queues=4, started=0, set_by_lib=0, split=0, env=None)),
    # HIP already initialised at 4 queues: nothing changes, the split stays off
    ({"ORBPL_ASSUME_RUNTIME_STARTED": "1", "GPU_MAX_HW_QUEUES": "4"},
     dict(queues=4, started=1, set_by_lib=0, split=0, env="4")),
    ({"ORBPL_ASSUME_RUNTIME_STARTED": "1", "GPU_MAX_HW_QUEUES": "4", "ORBPL_HW_QUEUES": "16"},
     dict(queues=4, started=1, set_by_lib=0, split=0, env="4")),
    ({"ORBPL_ASSUME_RUNTIME_STARTED": "1"}, dict(queues=4, started=1, set_by_lib=0, split=0, env=None)),
    # started with 16 queues: the split is on
    ({"ORBPL_ASSUME_RUNTIME_STARTED": "1", "GPU_MAX_HW_QUEUES": "16"},
     dict(queues=16, started=1, set_by_lib=0, split=1, env="16")),
    # the override still decides
    ({"GPU_MAX_HW_QUEUES": "4", "ORBPL_LSD_SPLIT": "1"},
     dict(queues=4, started=0, set_by_lib=0, split=1, env="4")),
])
def test_hw_queue_state(env, want):
    assert _state(**env) == want

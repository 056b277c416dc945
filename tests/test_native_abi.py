"""CPU-side checks of the C-ABI library (no GPU needed, no compute calls).

* liblbk8s.so loads and exports every function include/lbk8s.h declares;
* the ctypes structs match the header's field order (spot-checked by size);
* host-only entry points (config validation, state sizing) behave like the
  reference's constructor constraints.
"""
import ctypes as C
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "lbk8s.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(lb_\w+)\s*\(", src, re.M)))


def test_header_declares_expected_api():
    fns = declared_functions()
    for f in ("lb_init", "lb_reset", "lb_step", "lb_policy", "lb_state_bytes", "lb_last_error"):
        assert f in fns


def test_library_exports_every_declared_symbol():
    from lbk8s import _native
    L = _native.lib()
    for f in declared_functions():
        assert hasattr(L, f), f"{f} declared in include/lbk8s.h but not exported"
    assert set(declared_functions()) == set(_native.EXPORTED_SYMBOLS)
    assert L.lb_abi_version() == _native.ABI_VERSION


def test_struct_sizes_match_header_layout():
    from lbk8s import _native
    # 8 x int32 + 5 x double + uint64 + int64 + 2 x int32 = 32 + 40 + 16 + 8
    assert C.sizeof(_native.LBConfigC) == 96
    assert C.sizeof(_native.LBTraceC) == 15 * 8


def test_struct_offsets_match_compiled_header(tmp_path):
    """Every ctypes field offset equals offsetof() of the C compiler on include/lbk8s.h."""
    import subprocess

    from lbk8s import _native
    structs = {"lb_config": _native.LBConfigC, "lb_trace": _native.LBTraceC, "lb_ds_weights": _native.LBDSWeightsC,
               "lb_dqn_explore": _native.LBDQNExploreC}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "lbk8s.h"', "int main(void) {"]
    for cname, cls in structs.items():
        lines.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "off.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "off"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {tuple(l.split()[:2]): int(l.split()[2]) for l in out if l}
    for cname, cls in structs.items():
        assert got[(cname, "sizeof")] == C.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert got[(cname, f)] == getattr(cls, f).offset, (cname, f)


def test_geometry_is_a_config_field():
    """The E <= 8 kernel shape (and so the state layout) is chosen by lb_config.geometry."""
    from lbk8s import LBConfig, _native
    L = _native.lib()
    sizes = {}
    for g in ("auto", "tpe", "slice"):
        c = LBConfig().to_c(geometry=g)
        n = C.c_uint64()
        assert L.lb_state_bytes(C.byref(c), 4096, C.byref(n)) == 0
        sizes[g] = n.value
    assert sizes["auto"] == sizes["slice"] != sizes["tpe"]  # 4096 envs: lanes over endpoints
    c = LBConfig().to_c()
    c.geometry = 7
    assert L.lb_validate_config(C.byref(c)) != 0
    assert b"geometry" in L.lb_last_error()


def test_validate_and_state_bytes_host_only():
    from lbk8s import LBConfig, _native
    L = _native.lib()
    c = LBConfig().to_c()
    assert L.lb_validate_config(C.byref(c)) == 0
    n = C.c_uint64()
    assert L.lb_state_bytes(C.byref(c), 1 << 20, C.byref(n)) == 0
    # ~E*16 + ~100 bytes per env plus the lookup tables
    assert 100 * (1 << 20) < n.value < 400 * (1 << 20)
    bad = LBConfig().to_c()
    bad.num_nodes = 10
    assert L.lb_validate_config(C.byref(bad)) != 0
    assert b"IndexError" in L.lb_last_error()
    with pytest.raises(IndexError):
        _native.check(L.lb_validate_config(C.byref(bad)))


def test_config_mirrors_reference_constructor_errors():
    from lbk8s import LBConfig
    with pytest.raises(IndexError):
        LBConfig(num_nodes=12)
    with pytest.raises(IndexError):
        LBConfig(num_zones=3)
    with pytest.raises(TypeError):
        LBConfig(reward_function="bogus")
    c = LBConfig(num_endpoints=6, rejection_allowed=False)
    assert c.observation_space().shape == (6, 8)
    assert c.action_space().n == 6
    assert LBConfig().observation_space().shape == (9, 8)


def test_host_asan_ubsan_abi():
    """The C ABI's host code under AddressSanitizer + UBSan (tests/asan/abi_asan.cpp):
    validation, state-layout arithmetic, argument checks, error reporting, launch paths
    without a GPU (device code unsanitized: GPU sanitizers are not available on this pool)."""
    import shutil
    import subprocess
    if shutil.which("make") is None or not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("no hipcc / make")
    r = subprocess.run(["make", "-s", "-j6", "-C", os.path.join(REPO, "tests", "asan"), "run"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "abi_asan: ok" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr


def _rollout_kernel(B, steps, outputs_all=True, **kw):
    from lbk8s import LBConfig, _native
    L = _native.lib()
    to_c = {k: kw.pop(k) for k in ("geometry", "auto_reset") if k in kw}
    c = LBConfig(**kw).to_c(**to_c)
    k = C.c_int32(-1)
    assert L.lb_rollout_kernel(C.byref(c), B, steps, int(outputs_all), C.byref(k)) == 0, L.lb_last_error()
    return _native.LB_ROLLOUT[k.value]


def test_rollout_kernel_choice():
    """lb_rollout_kernel (host only): the bench's launch takes k_rollout_lean; shapes it does
    not cover fall back to k_rollout_img / k_rollout_tpe / the slice kernel."""
    assert _rollout_kernel(1 << 20, 20) == "k_rollout_lean_split"                 # the driver's launch
    assert _rollout_kernel(1 << 20, 100) == "k_rollout_lean"
    assert _rollout_kernel(2000 * 64, 100, num_endpoints=6, num_nodes=48, num_zones=12) == "k_rollout_lean"
    assert _rollout_kernel(1 << 20, 20, outputs_all=False) == "k_rollout_img"     # an output not written
    assert _rollout_kernel((1 << 20) + 1, 20) == "k_rollout_img"                  # a partial last wave
    assert _rollout_kernel(40000, 20, geometry="tpe") == "k_rollout_img"          # 64-thread blocks
    assert _rollout_kernel(1 << 20, 20, num_endpoints=7) == "k_rollout_img"       # E without a lean build
    assert _rollout_kernel(1 << 20, 20, reward_function="multi") == "k_rollout_lean_split"
    assert _rollout_kernel(1 << 20, 32) == "k_rollout_lean_split" and _rollout_kernel(1 << 20, 33) == "k_rollout_lean"
    assert _rollout_kernel(1 << 20, 120) == "k_rollout_tpe"                       # K > L: in-loop resets
    assert _rollout_kernel(1 << 20, 20, auto_reset=False) == "k_rollout_tpe"
    assert _rollout_kernel(1 << 20, 20, num_nodes=100) == "policy+step launches"
    assert _rollout_kernel(4096, 20) == "k_rollout_slice"
    assert _rollout_kernel(65536 + 320, 20, num_endpoints=6) == "k_rollout_lean_split"  # E = 6, N = 24: one zone word
    # lb_rollout's own preconditions hold here too: trace mode has no rollout kernel
    from lbk8s import LBConfig, _native
    c = LBConfig().to_c(trace=True)
    k = C.c_int32(-1)
    assert _native.lib().lb_rollout_kernel(C.byref(c), 1 << 20, 20, 1, C.byref(k)) != 0
    assert "Philox" in _native.lib().lb_last_error().decode()


def test_rollout_32bit_offsets_guard():
    """k_rollout_lean / k_rollout_img address with 32-bit byte offsets from scalar bases: a
    launch whose state blob, ep_stats rows or obs slot would pass 4 GiB takes the 64-bit
    k_rollout_tpe instead (an unguarded offset would wrap past 2^24 envs)."""
    from lbk8s import LBConfig, _native
    L = _native.lib()
    c = LBConfig().to_c()
    n = C.c_uint64()
    # the largest whole-wave B whose blob and obs slot stay below 4 GiB takes the lean kernel
    lo, hi = 1 << 16, 1 << 26
    while hi - lo > 64:
        mid = (lo + hi) // 2 // 64 * 64
        assert L.lb_state_bytes(C.byref(c), mid, C.byref(n)) == 0
        fits = n.value <= 0xFFFFFFFF and mid * 9 * 32 <= 0xFFFFFFFF and mid * 16 * 8 <= 0xFFFFFFFF
        lo, hi = (mid, hi) if fits else (lo, mid)
    assert _rollout_kernel(lo, 20) == "k_rollout_lean_split"
    big = lo + 64 * 4096
    assert _rollout_kernel(big, 20) == "k_rollout_tpe"
    assert _rollout_kernel(1 << 24, 20) == "k_rollout_tpe"       # 2^24 envs: ~6.6 GB of state
    assert _rollout_kernel((1 << 24) + 1, 20) == "k_rollout_tpe"


def test_library_built_from_tree_sources():
    """Build provenance: the in-tree liblbk8s.so embeds the SHA-256 of the sources it was
    compiled from (csrc/Makefile SRC_HASH), equal to the tree's; and the Makefile hashes the
    same files, in the same order, as the loader."""
    from lbk8s import _native
    L = _native.lib()
    assert L.lb_source_hash().decode() == _native.source_hash()
    mk = open(os.path.join(REPO, "gym-loadbalancing_amd", "csrc", "Makefile")).read()
    srcs = re.search(r"^SRCS := (.*?)(?<!\\)$", mk, re.S | re.M).group(1).replace("\\\n", " ").split()
    assert tuple(srcs) == _native.SOURCES


def _stub_library(tmp_path, flags):
    """A host-only stand-in for liblbk8s.so (gcc): every symbol the loader binds, the tree's
    source hash, the current ABI version and the given build flags."""
    import shutil
    import subprocess
    from lbk8s import _native
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    special = {"lb_abi_version", "lb_source_hash", "lb_build_flags", "lb_build_compiler", "lb_last_error"}
    lines = [f"int lb_abi_version(void) {{ return {_native.ABI_VERSION}; }}",
             f'const char* lb_source_hash(void) {{ return "{_native.source_hash()}"; }}',
             f'const char* lb_build_flags(void) {{ return "{flags}"; }}',
             'const char* lb_build_compiler(void) { return "stub"; }',
             'const char* lb_last_error(void) { return ""; }']
    lines += [f"int {f}(void) {{ return 0; }}" for f in _native.EXPORTED_SYMBOLS if f not in special]
    src = tmp_path / "stub.c"
    src.write_text("\n".join(lines) + "\n")
    out = tmp_path / "liblbk8s_stub.so"
    subprocess.run(["gcc", "-shared", "-fPIC", "-o", str(out), str(src)], check=True)
    return str(out)


def _load_as_product(monkeypatch, path):
    from lbk8s import _native
    monkeypatch.setattr(_native, "LIB_PATH", path)
    monkeypatch.setattr(_native, "_PRODUCT_LIB", path)
    monkeypatch.setattr(_native, "_lib", None)
    return _native.lib()


def test_loader_refuses_knob_build(tmp_path, monkeypatch):
    """Build provenance covers the flags, not only the sources: a product library carrying the
    tree's source hash but compiled with a diagnostic -D knob (-DLB_LEAN_ST_AUX=18, the obs
    stores' cache policy) is refused by _native.lib(); the same stand-in with the Makefile's
    default flags loads."""
    from lbk8s import _native
    want = _native.expected_build_flags()
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    ok = _stub_library(tmp_path / "a", want)
    assert _load_as_product(monkeypatch, ok).lb_build_flags().decode() == want
    bad = _stub_library(tmp_path / "b", want + " -DLB_LEAN_ST_AUX=18")
    with pytest.raises(_native.NonDefaultBuild, match="LB_LEAN_ST_AUX=18"):
        _load_as_product(monkeypatch, bad)


def test_makefile_embeds_build_flags():
    """csrc/Makefile compiles its flags, -D defines included, into the library (lb_build_flags):
    a DEFS knob appears in the embedded string, so the loader sees it; and the in-tree product
    library carries exactly the defaults."""
    import shutil
    import subprocess
    from lbk8s import _native
    if shutil.which("make") is None:
        pytest.skip("no make")
    csrc = os.path.join(REPO, "gym-loadbalancing_amd", "csrc")
    r = subprocess.run(["make", "-n", "-B", "-C", csrc, "DEFS=-DLB_LEAN_ST_AUX=18"], capture_output=True, text=True,
                       check=True)
    line = [x for x in r.stdout.splitlines() if "LBK8S_BUILD_FLAGS" in x][0]
    embedded = re.search(r"-DLBK8S_BUILD_FLAGS='\"([^\"]*)\"'", line).group(1)
    assert embedded == _native.expected_build_flags() + " -DLB_LEAN_ST_AUX=18"
    L = _native.lib()
    assert L.lb_build_flags().decode() == _native.expected_build_flags()
    assert "clang version" in L.lb_build_compiler().decode()


def test_dqn_one_launch_shape_is_device_independent():
    """lb_dqn_steps_supported (host only) depends on the env's shape alone -- the slice layout
    with 16 lanes per env and R <= 16 -- not on the device's CU count (gated on
    occupancy, a part with more CUs would have sent the learner to the three-launch path):
    from run.py's 8 envs to config 5's 4096, and not for the thread-per-env layout or R > 16."""
    from lbk8s import LBConfig, _native
    L = _native.lib()
    c = LBConfig().to_c()
    for B in (1, 8, 64, 4096, 4104, 32767):
        assert L.lb_dqn_steps_supported(C.byref(c), B, 9) == 1, B
    assert L.lb_dqn_steps_supported(C.byref(c), 65536, 9) == 0          # thread-per-env layout
    c6 = LBConfig(num_endpoints=6, num_nodes=48, num_zones=12, reward_function="multi").to_c()
    assert L.lb_dqn_steps_supported(C.byref(c6), 8, 7) == 1            # run.py's own setup
    c20 = LBConfig(num_endpoints=20).to_c()
    assert L.lb_dqn_steps_supported(C.byref(c20), 4096, 21) == 0        # R > 16

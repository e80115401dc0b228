"""Host AddressSanitizer + UndefinedBehaviorSanitizer run of the C-ABI argument checking
(SURVEY §5 "Host ASan on the C-ABI shim").

The library's translation units are compiled host-only (`--offload-host-only`: no device
code, so no GPU is needed and the build takes seconds) with -fsanitize=address,undefined,
linked against tests/asan/hip_stubs.cpp (a stand-in HIP runtime whose device operations fail
and are counted) and tests/asan/abi_args.cpp, which drives every codec_* entry of include/codec_tcc.h
with NULL pointers, bad shapes, overflowing sizes and short workspaces.  Every call must
return its negative status (or 0 bytes) with no sanitizer report.  GPU sanitizers are not
available on this pool; this covers the host side only."""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
SAN = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"]


@pytest.fixture(scope="module")
def abi_args_binary(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not installed")
    from codec_tcc_amd import build
    out = tmp_path_factory.mktemp("asan")
    objs = []
    jobs = []
    for src in build.SRCS:
        obj = str(out / (os.path.basename(src) + ".o"))
        cmd = [HIPCC, "-O1", "-g", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--offload-host-only", *SAN,
               f"-I{build.INC}", "-c", src, "-o", obj]
        jobs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
        objs.append(obj)
    for p in jobs:
        _o, err = p.communicate()
        assert p.returncode == 0, err[-4000:]
    # the host-only objects still name their (absent) code objects: give them empty ones
    nm = subprocess.run(["nm", "-u", *objs], capture_output=True, text=True, check=True).stdout
    fatbins = sorted(set(re.findall(r"\b(__hip_fatbin_[0-9a-f]+)\b", nm)))
    dig = out / "digest.cpp"
    dig.write_text('extern "C" const char* codec_build_digest(void) { return "asan-host-build"; }\n' +
                   "".join(f'extern "C" {{ char {f}[64]; }}\n' for f in fatbins))
    for src in (os.path.join(REPO, "tests", "asan", "abi_args.cpp"), os.path.join(REPO, "tests", "asan", "hip_stubs.cpp"),
                str(dig)):
        obj = str(out / (os.path.basename(src) + ".o"))
        r = subprocess.run([HIPCC, "-O1", "-g", "-std=c++17", "--offload-arch=gfx950", "--offload-host-only", *SAN,
                            f"-I{build.INC}", "-c", src, "-o", obj], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-4000:]
        objs.append(obj)
    exe = str(out / "abi_args")
    # linked with clang++ against the stubs only (no libamdhip64, so no GPU runtime at all)
    r = subprocess.run(["/opt/rocm/lib/llvm/bin/clang++", *SAN, *objs, "-o", exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    return exe


def test_c_abi_rejects_bad_arguments_under_asan(abi_args_binary):
    env = dict(os.environ,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:verify_asan_link_order=0:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               HIP_VISIBLE_DEVICES="")
    r = subprocess.run([abi_args_binary], capture_output=True, text=True, timeout=300, env=env)
    report = r.stdout + r.stderr
    assert "AddressSanitizer" not in report and "runtime error" not in report, report[-6000:]
    assert r.returncode == 0, report[-6000:]
    m = re.search(r"abi_args: (\d+) calls, 0 failures", r.stdout)
    assert m and int(m.group(1)) > 300, report[-3000:]


def test_every_header_entry_is_driven():
    """abi_args.cpp calls every function include/codec_tcc.h declares."""
    hdr = open(os.path.join(REPO, "include", "codec_tcc.h")).read()
    declared = set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(codec_\w+)\s*\(", hdr, re.M))
    src = open(os.path.join(REPO, "tests", "asan", "abi_args.cpp")).read()
    called = set(re.findall(r"\b(codec_\w+)\s*\(", src))
    assert declared <= called, sorted(declared - called)


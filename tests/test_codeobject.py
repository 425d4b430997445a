"""Register budget of the built gfx950 code object (CPU tier: reads the kernel
metadata of kvecc/libkvecc.so, launches nothing).

Occupancy regressions are silent in the parity tests: in round 2 one extra
condition took the interpolating fused read from 128 to 131 VGPRs, below the
2 workgroups per CU its grid assumes, and the kernel ran 20 % slower.  These
checks pin what the launches assume:
- no product kernel spills registers or uses scratch;
- the fused-read tile kernels for fp16/bf16 output (the shim's dtypes) fit
  128 VGPRs: 2 x 512-thread workgroups per CU (KVECC_SHIM_TILE_PER_CU);
- the bench's headline decode and the per-head row kernels stay within their
  measured budgets.
Skipped when the ROCm LLVM tools or the built library are absent.
"""

import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd", "kvecc", "libkvecc.so")
LLVM = "/opt/rocm/lib/llvm/bin"
TOOLS = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf")]


@pytest.fixture(scope="module")
def kernels(tmp_path_factory):
    if not os.path.exists(LIB) or not all(os.path.exists(t) for t in TOOLS):
        pytest.skip("libkvecc.so or the ROCm LLVM tools are missing")
    d = tmp_path_factory.mktemp("co")
    fat = str(d / "fatbin.bin")
    subprocess.run([TOOLS[0], f"--dump-section=.hip_fatbin={fat}", LIB, str(d / "lib.stripped")], check=True)
    # one offload bundle per translation unit, concatenated in the section
    with open(fat, "rb") as f:
        blob = f.read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), blob)]
    notes = ""
    for i, st in enumerate(starts):
        part, co = str(d / f"b{i}.bin"), str(d / f"b{i}.o")
        with open(part, "wb") as f:
            f.write(blob[st:starts[i + 1] if i + 1 < len(starts) else len(blob)])
        subprocess.run([TOOLS[1], "--unbundle", "--type=o", f"--input={part}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes += subprocess.run([TOOLS[2], "--notes", co], check=True, capture_output=True, text=True).stdout
    out = {}
    for ent in re.split(r"\n\s+- \.agpr_count:", notes)[1:]:
        field = lambda k: re.search(rf"\.{k}:\s+(\S+)", ent)  # noqa: E731
        if field("name") is None or field("vgpr_count") is None:
            continue
        out[field("name").group(1)] = {
            "lds": int(field("group_segment_fixed_size").group(1)),
            "block": int(field("max_flat_workgroup_size").group(1)),
            "vgpr": int(field("vgpr_count").group(1)),
            "agpr": int(ent.split("\n", 1)[0].strip()),
            "spill": int(field("vgpr_spill_count").group(1)) if field("vgpr_spill_count") else 0,
            "scratch": int(field("private_segment_fixed_size").group(1)),
        }
    shutil.rmtree(d, ignore_errors=True)
    assert out, "no kernel metadata found"
    return out


def test_no_spills_or_scratch(kernels):
    bad = {k: v for k, v in kernels.items() if v["spill"] or v["scratch"]}
    assert not bad, bad


def test_fused_read_tiles_fit_two_workgroups_per_cu(kernels):
    # shim_read_{bytes,golay}_tiles_kernel / shim_read_h84_interp_kernel <__half | __hip_bfloat16, ...>
    tiles = {k: v for k, v in kernels.items()
             if re.search(r"shim_read_((bytes|golay)_tiles|h84_interp)_kernelI(6__half|14__hip_bfloat16)", k)}
    assert len(tiles) >= 24, sorted(tiles)
    over = {k: v["vgpr"] for k, v in tiles.items() if v["vgpr"] + v["agpr"] > 128}
    assert not over, over


@pytest.mark.parametrize("pattern,limit", [
    (r"^_ZN5kvecc19golay_decode_kernel", 64),       # the headline decode
    (r"^_ZN5kvecc19golay_encode_kernel", 64),
    (r"golay_decode_rows_reg_kernel", 128),         # per-head rows decode (256 threads, 3 per CU)
    (r"golay_encode_rows_full_kernel", 64),         # per-head rows encode (full grid)
])
def test_hot_kernel_budgets(kernels, pattern, limit):
    hit = {k: v["vgpr"] + v["agpr"] for k, v in kernels.items() if re.search(pattern, k)}
    assert hit, pattern
    assert max(hit.values()) <= limit, hit


# The tuned launch shapes the library ships (csrc/*.hip constants).
# Each kernel's static LDS and workgroup size are fixed by those constants, so a
# build with other values (an experiment's) fails here.
SHIPPED = [
    # fused Golay read: 256 threads, 32 KiB tables + 4 x (2304 B tile + 256 B scales)
    (r"shim_read_golay_tiles_kernelI6__half", 256, 32768 + 4 * (2304 + 256)),
    # fused byte-codec read: 128 threads (2 independent waves), 2 x (2304 + 256) B
    (r"shim_read_bytes_tiles_kernelI6__half", 128, 2 * (2304 + 256)),
    # interpolating H(8,4) read: 128 threads (2 independent waves), 2 x (2304 + 256) B
    (r"shim_read_h84_interp_kernelI6__half", 128, 2 * (2304 + 256)),
    # packed Golay decode wave tiles: 512 threads, 24 KiB tables + 8 x 3 KiB stage
    (r"golay_decode_packed_wave_kernel", 512, 24576 + 8 * 3072),
    # per-head rows register tiles: 512 threads
    (r"golay_decode_rows_reg_kernelILb1ELi256ELj30E", 256, None),
    # per-head rows encode on a full grid: 512 threads, split parity (256 B) + 8 x 2816 B codeword tiles
    (r"golay_encode_rows_full_kernel", 512, 256 + 8 * 2816),
    (r"^_ZN5kvecc19golay_decode_kernel", 512, None),
    (r"^_ZN5kvecc19golay_encode_kernel", 1024, None),
]


@pytest.mark.parametrize("pattern,block,lds", SHIPPED)
def test_shipped_launch_shapes(kernels, pattern, block, lds):
    hit = {k: v for k, v in kernels.items() if re.search(pattern, k)}
    assert hit, pattern
    for k, v in hit.items():
        assert v["block"] == block, (k, v)
        if lds is not None:
            assert v["lds"] == lds, (k, v)


def test_no_experiment_switches_in_product_sources():
    """The product sources carry no build-time switches (#if/#ifndef KVECC_*):
    experiment variants live in tools/exp forks, so no -D can change what the
    library computes.  The only KVECC_ preprocessor guard left is kvecc.h's own
    include guard."""
    csrc = os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd", "csrc")
    bad = []
    for f in sorted(os.listdir(csrc)):
        for i, line in enumerate(open(os.path.join(csrc, f)), 1):
            if re.match(r"\s*#\s*(if|ifdef|ifndef|elif)\b.*\bKVECC_", line):
                bad.append(f"{f}:{i}: {line.strip()}")
    assert not bad, bad


def test_no_experiment_symbols_exported():
    """libkvecc.so exports the C ABI of include/kvecc.h and nothing from the
    experiment forks (kvecc_exp_*) or the round-3 wave-timing probe."""
    readelf = os.path.join(LLVM, "llvm-readelf")
    if not os.path.exists(LIB) or not os.path.exists(readelf):
        pytest.skip("libkvecc.so or llvm-readelf missing")
    syms = subprocess.run([readelf, "--dyn-syms", "-W", LIB], check=True, capture_output=True, text=True).stdout
    assert "kvecc_golay_decode" in syms  # the C ABI is there
    bad = [ln for ln in syms.splitlines() if "kvecc_exp_" in ln or "wave_times" in ln]
    assert not bad, bad

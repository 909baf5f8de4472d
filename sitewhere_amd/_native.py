"""Build and load the native libraries of SiteWhere-AMD.

Two shared objects are built **in-tree** under ``sitewhere_amd/_lib``:

* ``libswnative.so`` (g++): the host runtime -- partitioned commit log
  (Kafka replacement), registry builder, CPU batch decoder, fleet generator,
  and the multi-threaded native CPU engine shard (``swce_*``).
* ``libswgpu.so`` (hipcc ``--offload-arch=gfx950``): the CDNA4 data-plane kernels.

Both expose a plain C ABI and are loaded with :mod:`ctypes`; there is no
hipify step and no torch C++ ABI dependency.  ``libswgpu.so`` links the HIP
runtime by soname (``libamdhip64.so.7``); torch must be imported first so the
process uses torch's already-loaded runtime (one HIP runtime per process).
"""
from __future__ import annotations

import ctypes
import os
import shutil
import subprocess
import threading
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
LIB_DIR = Path(__file__).resolve().parent / "_lib"
CSRC = ROOT / "csrc"
GPU_ARCH = os.environ.get("SW_GPU_ARCH", "gfx950")

_NATIVE_SRC = [CSRC / "native" / "swnative.cpp", CSRC / "native" / "swcpuengine.cpp", CSRC / "native" / "swseg.cpp",
               CSRC / "native" / "swindex.cpp", CSRC / "native" / "swroute.cpp", CSRC / "native" / "swsandbox.cpp", CSRC / "native" / "swjson.cpp",
               CSRC / "native" / "swrowjson.cpp"]
_GPU_SRC = [CSRC / "hip" / "swgpu.hip", CSRC / "hip" / "swseg.hip", CSRC / "hip" / "swindex.hip"]
_HEADERS = sorted((CSRC / "include").glob("*.h"))

_lock = threading.Lock()
_native = None
_gpu = None


class NativeBuildError(RuntimeError):
    pass


def _stale(target: Path, sources) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(s.stat().st_mtime > t for s in list(sources) + _HEADERS)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise NativeBuildError(f"build failed: {' '.join(map(str, cmd))}\n{r.stdout}\n{r.stderr}")


def build_native(force: bool = False) -> Path:
    """Compile libswnative.so with g++ (C++17, -O3)."""
    LIB_DIR.mkdir(parents=True, exist_ok=True)
    out = LIB_DIR / "libswnative.so"
    if force or _stale(out, _NATIVE_SRC):
        cxx = shutil.which("g++") or shutil.which("c++") or "g++"
        tmp = out.with_suffix(".so.tmp")
        _run([cxx, "-O3", "-std=c++17", "-shared", "-fPIC", f"-I{CSRC / 'include'}", "-o", str(tmp),
              *map(str, _NATIVE_SRC), "-lpthread"])
        os.replace(tmp, out)
    return out


def hipcc_path() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise NativeBuildError("hipcc not found (ROCm is required to build the gfx950 kernels)")


def build_gpu(force: bool = False) -> Path:
    """Cross-compile libswgpu.so for gfx950 with hipcc (works without a GPU)."""
    LIB_DIR.mkdir(parents=True, exist_ok=True)
    out = LIB_DIR / "libswgpu.so"
    if force or _stale(out, _GPU_SRC):
        tmp = out.with_suffix(".so.tmp")
        _run([hipcc_path(), f"--offload-arch={GPU_ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC",
              f"-I{CSRC / 'include'}", "-o", str(tmp), *map(str, _GPU_SRC), "-lhsa-runtime64"])
        os.replace(tmp, out)
    return out


def build_all(force: bool = False):
    return build_native(force), build_gpu(force)


# ----------------------------------------------------------------------------- prototypes
c_void_p, c_int32, c_int64, c_uint64, c_double, c_char_p = (
    ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double, ctypes.c_char_p)


def _proto(lib, name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)


def native():
    """Load (building if needed) the host runtime library."""
    global _native
    if _native is not None:
        return _native
    with _lock:
        if _native is not None:
            return _native
        path = LIB_DIR / "libswnative.so"
        if _stale(path, _NATIVE_SRC):
            build_native()
        lib = ctypes.CDLL(str(path))
        P = c_void_p
        _proto(lib, "sw_fingerprint_batch", None, P, P, c_int64, P, P)
        _proto(lib, "sw_hash64_batch", None, P, P, c_int64, P)
        _proto(lib, "sw_hash64_ranges", None, P, P, P, c_int64, P)
        _proto(lib, "sw_murmur2", c_int32, P, c_int32)
        _proto(lib, "sw_crc32c", ctypes.c_uint32, ctypes.c_char_p, c_int64)
        _proto(lib, "sw_memcpy_mt", None, P, P, c_int64, c_int32)
        _proto(lib, "sw_partition_for_key", c_int32, P, c_int32, c_int32)
        _proto(lib, "sw_partition_payloads", None, P, P, c_int64, c_int32, P)
        _proto(lib, "sw_reg_upsert", c_int64, P, P, P, c_int64, c_uint64, c_uint64, c_int32)
        _proto(lib, "sw_reg_find", c_int64, P, P, P, c_int64, c_uint64, c_uint64)
        _proto(lib, "sw_reg_build", c_int64, P, P, P, c_int64, P, P, P, c_int64, P)
        _proto(lib, "sw_cpu_decode", c_int64, P, P, c_int64, c_int64, c_int32, P, P, c_int64, c_int32)
        _proto(lib, "sw_gen_payloads", c_int64, c_int64, c_char_p, c_int64, c_double, c_double, c_double, c_int32,
               c_int32, c_int64, c_uint64, c_int32, c_double, c_double, c_double, c_double, P, c_int64, P,
               c_uint64)
        _proto(lib, "sw_gen_tokens", c_int64, c_char_p, c_int64, c_int64, P, c_int64, P)
        _proto(lib, "sw_stamp_alt_epoch", c_int64, P, P, c_int64, c_uint64, c_int32)
        _proto(lib, "sw_alt_positions", c_int64, P, P, c_int64, P)
        _proto(lib, "sw_stamp_positions", c_int64, P, P, c_int64, c_uint64, c_int32)
        _proto(lib, "sw_json_to_pb", c_int64, P, c_int64, P, c_int64)
        _proto(lib, "sw_json_to_pb_batch", c_int64, P, P, c_int64, P, c_int64, P, P)
        _proto(lib, "swlog_open", P, c_char_p, c_int32)
        _proto(lib, "swlog_close", None, P)
        _proto(lib, "swlog_topic", c_int32, P, c_char_p, c_int32)
        _proto(lib, "swlog_partitions", c_int32, P, c_int32)
        _proto(lib, "swlog_append_batch", c_int64, P, c_int32, c_int32, P, P, P, P, P, c_int64)
        _proto(lib, "swlog_append_routed", c_int64, P, P, P, c_int64, P, P, c_int64, P)
        _proto(lib, "swlog_append", c_int64, P, c_int32, c_int32, P, c_int64, P, c_int64, c_int64)
        _proto(lib, "swlog_end_offset", c_int64, P, c_int32, c_int32)
        _proto(lib, "swlog_begin_offset", c_int64, P, c_int32, c_int32)
        _proto(lib, "swlog_bytes_from", c_int64, P, c_int32, c_int32, c_int64)
        _proto(lib, "swlog_wait", c_int64, P, c_int32, c_int32, c_int64, c_int32)
        _proto(lib, "swlog_read", c_int64, P, c_int32, c_int32, c_int64, c_int64, P, c_int64, P)
        _proto(lib, "swlog_retain_from", c_int64, P, c_int32, c_int32, c_int64)
        _proto(lib, "swlog_commit", c_int32, P, c_char_p, c_int32, c_int32, c_int64)
        _proto(lib, "swlog_committed", c_int64, P, c_char_p, c_int32, c_int32)
        _proto(lib, "swlog_flush", c_int32, P)
        _proto(lib, "swlog_set_retention", c_int32, P, c_int32, c_int64)
        _proto(lib, "swlog_take_released", c_int64, P, P, c_int64)
        # native CPU engine shard (csrc/native/swcpuengine.cpp)
        _proto(lib, "swce_create", P, c_int32)
        _proto(lib, "swce_destroy", None, P)
        _proto(lib, "swce_threads", c_int32, P)
        _proto(lib, "swce_reserve", None, P, c_int64, c_int64)
        _proto(lib, "swce_capture_names", c_int64, P, P, c_int64, P, c_int64)
        _proto(lib, "swce_process", c_int32, P, P, P, P, c_int64, c_int64, c_int32, P, P, P, P, P)
        for kind in ("dedup", "intern", "seen", "ms"):
            _proto(lib, f"swce_{kind}_size", c_int64, P)
        _proto(lib, "swce_dedup_export", c_int64, P, P, P)
        _proto(lib, "swce_dedup_window", None, P, c_int64, c_int64)
        _proto(lib, "swce_ff_init", c_int32, P, c_int64, c_int64, c_int64)
        _proto(lib, "swce_ff_add", None, P, c_int64, P, c_int64)
        _proto(lib, "swce_ff_clear", None, P, c_int64)
        _proto(lib, "swce_ff_meta", None, P, P, P)
        _proto(lib, "swce_ff_export", c_int64, P, P, P, c_int64)
        _proto(lib, "swce_ff_import", c_int32, P, P, P, c_int64)
        _proto(lib, "swce_dedup_prev_size", c_int64, P)
        _proto(lib, "swce_dedup_prev_export", c_int64, P, P, P)
        _proto(lib, "swce_dedup_prev_import", None, P, P, P, c_int64)
        _proto(lib, "swce_dedup_import", None, P, P, P, c_int64)
        _proto(lib, "swce_intern_export", c_int64, P, P, P)
        _proto(lib, "swce_intern_import", None, P, P, P, c_int64)
        _proto(lib, "swce_seen_export", c_int64, P, P)
        _proto(lib, "swce_seen_import", None, P, P, c_int64)
        _proto(lib, "swce_ms_export", c_int64, P, P)
        _proto(lib, "swce_ms_import", None, P, P, c_int64)
        _proto(lib, "swce_ms_of", c_int64, P, c_int32, P, c_int64)
        # durable columnar segments (csrc/native/swseg.cpp)
        _proto(lib, "swseg_encode", c_int64, P, P, P, P, c_int64, c_int64, P, c_int64)
        _proto(lib, "swseg_seal", None, P, c_int64, c_int64, c_int64, c_int32, c_int32)
        _proto(lib, "swseg_verify", c_int32, P, c_int64)
        _proto(lib, "swseg_verify_pages", c_int32, P, c_int64, c_int64, c_int64)
        _proto(lib, "swseg_decode", c_int64, P, c_int64, c_int64, P, P, P, P, P, P, P, P, P, P, c_int64, P)
        _proto(lib, "swseg_alt_page_rows", c_int64, P, P, P, P, P, c_int64, c_int32, P, P, c_int64, P)
        _proto(lib, "swseg_fetch_rows", c_int64, P, P, P, P, P, c_int64, c_int32, P, P, P, P, P, P, P, P, P, P,
               c_int64, P, P)
        _proto(lib, "swseg_string_bytes", c_int64, P, c_int64, c_int64)
        _proto(lib, "swseg_page_summary", c_int64, P, P)
        _proto(lib, "swseg_index_block", c_int64, P, c_int64, P, P, P, P, P, P)
        _proto(lib, "swseg_multi_range_u64", None, P, P, c_int64, c_uint64, P, P)
        _proto(lib, "swseg_multi_find_u64", None, P, P, c_int64, P, c_int64, P, P)
        _proto(lib, "swseg_multi_range_u32", None, P, P, P, P, c_int64, ctypes.c_uint32, c_int64, c_int64, P, P)
        _proto(lib, "swseg_dates", None, P, P, P)
        # block index trailers (csrc/native/swindex.cpp, format csrc/include/swindex.h)
        _proto(lib, "swseg_index_append", c_int64, P, c_int64, P, c_int64)
        _proto(lib, "swseg_ix_verify", c_int32, P, c_int64, c_int64, c_int64)
        _proto(lib, "swseg_ix_offset", c_int64, P)
        _proto(lib, "swseg_ix_max_bytes", c_int64, c_int64)
        _proto(lib, "swseg_ix_alt_pages", c_int64, P, c_int64, c_uint64, P, P, c_int64)
        _proto(lib, "swseg_ix_alt_find", None, P, c_int64, P, c_int64, P, P)
        _proto(lib, "swseg_ix_asg_pages", c_int64, P, c_int64, c_int32, c_int64, c_int64, P, P, c_int64)
        _proto(lib, "swseg_ix_asgs_pages", c_int64, P, c_int64, P, c_int64, P, c_int64, c_int64, P, P, c_int64, P, P, P)
        _proto(lib, "swseg_ix_ctx_find", None, P, c_int64, c_int32, ctypes.c_uint32, P)
        _proto(lib, "swseg_image_addrs", None, P, P, P, c_int64, P)
        _proto(lib, "swseg_rechecksum", None, P)
        _proto(lib, "swseg_alt_hashes", c_int64, P, P, c_int64)
        _proto(lib, "swseg_scan_pages", c_int64, P, P, P, P, P, c_int64, c_int32, c_int32, P, c_int64, c_int32,
               c_int64, c_int64, c_int32, P, P, P, c_int64, P, P, P, P, P)
        _proto(lib, "swss_open", P, c_char_p, c_int32, c_int64, c_int64, c_int32)
        _proto(lib, "swss_append", c_int32, P, P, c_int64, c_int64)
        _proto(lib, "sw_varint_offsets", c_int32, P, c_int64, c_int64, c_int64, P)
        _proto(lib, "swss_append_commit", c_int32, P, P, c_int64, c_int64, P, P, c_int32)
        _proto(lib, "swss_sources", c_int64, P, P, P, c_int64)
        _proto(lib, "swseg_set_flags", None, P, c_int32)
        _proto(lib, "swss_durable", c_int64, P)
        _proto(lib, "swss_error", c_int32, P)
        _proto(lib, "swss_wait", c_int32, P, c_int64, c_int64)
        _proto(lib, "swjson_rows", c_int64, P, c_int64, P, P, P, P, P, P, P, P, P, P, P,
               c_int64, c_int64, c_int64, c_int64, c_int64, c_int64, P, P, P, c_int64, P, P, P, c_int64, P, P, P,
               P, c_int64, P, c_int64, P, P, c_int64, P, P)
        _proto(lib, "swjson_select_block", c_int64, P, c_int32, P, c_int64, c_int32, P, c_int64, P, P, P, P, P, P,
               c_int64, P, P, P, P, c_int64, c_int32, P, c_int64, P, c_int64, P, c_int64, P, P, c_int64, P, P, P,
               c_int64)
        _proto(lib, "swseg_threshold_rows", c_int64, P, P, c_int64, ctypes.c_double, ctypes.c_double, c_int32,
               c_int32, c_int32, P, P, P, c_int64)
        _proto(lib, "swmqtt_scan", c_int64, P, c_int64, P, c_int64, c_int64, P)
        _proto(lib, "swmqtt_qos0_topics", c_int64, P, P, c_int64, P, c_int64, P)
        _proto(lib, "swmqtt_publish_qos0", c_int64, P, P, P, P, c_int64, ctypes.c_uint8, P, c_int64)
        _proto(lib, "swss_stats", None, P, P)
        _proto(lib, "swss_set_retention", None, P, c_int64, c_int64, c_int64)
        _proto(lib, "swss_close", None, P)
        _proto(lib, "swss_index", c_int64, P, P, c_int64)
        _proto(lib, "swss_index_tr", c_int64, P, P, P, P, P, c_int64)
        _proto(lib, "swss_mem_caps", c_int64, P, c_int64, c_int64, P)
        _proto(lib, "swss_lease_begin", c_int64, P)
        _proto(lib, "swss_lease_end", None, P, c_int64)
        _proto(lib, "swseg_ix_page_geom", c_int64, P, c_int64, P, P, c_int64, P, P)
        _proto(lib, "swseg_ix_ctx_heads", c_int64, P, c_int64, c_int32, ctypes.c_uint32, P, P, P, P, c_int64)
        _proto(lib, "swss_file", c_int32, P, c_int32, c_char_p, c_int32)
        _proto(lib, "sw_route_rejects", c_int64, P, P, c_int64, P, P, c_int64, c_char_p, P, P, c_int64, P,
               c_int64, P, c_int64, P, P)
        _proto(lib, "sw_route_refs", c_int64, P, P, P, c_int64, c_int32, c_char_p, P, P, c_int64, P, c_int64, P,
               c_int64, P, P)
        _native = lib
        return lib


_native_gil = None


def native_gil():
    """The host runtime library bound with ``ctypes.PyDLL``: calls keep the GIL.

    For the bus's microsecond calls (append, read, offsets, commit).  Through ``CDLL`` every such
    call releases the GIL and must win it back from the busy service threads -- measured at
    0.1-1 ms per call on the per-event path (a convoy), for 4-80 us of native work."""
    global _native_gil
    if _native_gil is not None:
        return _native_gil
    lib0 = native()
    with _lock:
        if _native_gil is None:
            lib = ctypes.PyDLL(lib0._name)
            P = c_void_p
            _proto(lib, "swlog_topic", c_int32, P, c_char_p, c_int32)
            _proto(lib, "swlog_partitions", c_int32, P, c_int32)
            _proto(lib, "swlog_append_batch", c_int64, P, c_int32, c_int32, P, P, P, P, P, c_int64)
            _proto(lib, "swlog_append_routed", c_int64, P, P, P, c_int64, P, P, c_int64, P)
            _proto(lib, "swlog_append", c_int64, P, c_int32, c_int32, P, c_int64, P, c_int64, c_int64)
            _proto(lib, "swlog_end_offset", c_int64, P, c_int32, c_int32)
            _proto(lib, "swlog_begin_offset", c_int64, P, c_int32, c_int32)
            _proto(lib, "swlog_read", c_int64, P, c_int32, c_int32, c_int64, c_int64, P, c_int64, P)
            _proto(lib, "swlog_commit", c_int32, P, c_char_p, c_int32, c_int32, c_int64)
            _proto(lib, "swlog_committed", c_int64, P, c_char_p, c_int32, c_int32)
            _proto(lib, "swlog_append_external", c_int64, P, c_int32, c_int32, P, c_int64, c_int64, c_int64,
                   c_int64)
            _proto(lib, "swlog_view", c_int32, P, c_int32, c_int32, c_int64, P, P, P)
            _proto(lib, "swlog_hold", c_int32, P, c_int32, c_int32, c_int64)
            _proto(lib, "swlog_take_released", c_int64, P, P, c_int64)
            _proto(lib, "sw_partition_for_key", c_int32, c_char_p, c_int32, c_int32)
            _native_gil = lib
    return _native_gil


def gpu():
    """Load the gfx950 kernel library.  Raises if it is missing -- never falls back silently."""
    global _gpu
    if _gpu is not None:
        return _gpu
    import torch  # noqa: F401  -- one HIP runtime per process: torch's, loaded first

    with _lock:
        if _gpu is not None:
            return _gpu
        override = os.environ.get("SW_GPU_LIB")       # an experiment build (e.g. scripts/build_xcd_variant.sh)
        path = Path(override) if override else LIB_DIR / "libswgpu.so"
        if not override and _stale(path, _GPU_SRC):
            build_gpu()
        lib = ctypes.CDLL(str(path))
        P = c_void_p
        _proto(lib, "sw_phase_decode", c_int32, P, P)
        _proto(lib, "sw_phase_partition", c_int32, P, P)
        _proto(lib, "sw_phase_unpack", c_int32, P, P)
        _proto(lib, "sw_phase_process", c_int32, P, P, P)
        _proto(lib, "sw_registry_patch", c_int32, P, P, P, c_int64, P)
        _proto(lib, "sw_pip_batch", c_int32, P, c_int64, P, P, c_int64, P, P)
        _proto(lib, "sw_store_filter", c_int32, P, P, P, c_int64, c_int32, P, c_int64, c_int64, c_int64, P, c_int64,
               P, P)
        _proto(lib, "sw_scan_u32", c_int32, P, c_int64, P, P, P, c_int64, P)
        _proto(lib, "sw_state_lookup", c_int32, P, c_int64, c_int32, c_int32, P, P, P)
        _proto(lib, "sw_abi_sizes", c_int32, P)
        _proto(lib, "sw_host_alloc", c_int32, c_int64, P, P)
        _proto(lib, "sw_host_free", c_int32, P)
        _proto(lib, "sw_push_out", c_int32, P, P, P, c_int64, c_int32, P)
        _proto(lib, "sw_copy_d2h", c_int32, P, P, c_int64, P)
        _proto(lib, "sw_sdma_copy", c_int32, P, P, c_int64, c_int32, ctypes.POINTER(ctypes.c_uint64))
        _proto(lib, "sw_sdma_h2d", c_int32, P, P, c_int64, c_int32, ctypes.POINTER(ctypes.c_uint64))
        _proto(lib, "sw_frame_varint", c_int32, P, c_int64, c_int64, P, ctypes.c_uint32, P, c_int64, P)
        _proto(lib, "sw_set_step_params", c_int32, P, c_int64, c_int64, c_int64, P, P, c_int64, P)
        _proto(lib, "sw_graph_capture_process", c_int32, P, P, c_int32, P, ctypes.POINTER(ctypes.c_void_p))
        _proto(lib, "sw_graph_launch", c_int32, P, P)
        _proto(lib, "sw_graph_destroy", c_int32, P)
        _proto(lib, "sw_sdma_wait", c_int32, c_uint64)
        _proto(lib, "sw_seg_encode", c_int32, P, P, P, P, P, c_int64, P, c_int64, P)
        _proto(lib, "sw_seg_encode_stamped", c_int32, P, P, P, P, P, c_int64, P, c_int64, P, P)
        _proto(lib, "sw_seg_encode_snap", c_int32, P, P, P, P, P, c_int64, P, c_int64, P, P, P, P, P)
        _proto(lib, "sw_seg_aux", c_int32, P, P, P, P, P, c_int64, P, P, c_int64, P)
        # block index trailers + the radix sort (csrc/hip/swindex.hip)
        _proto(lib, "sw_radix_tmp_words", c_int64, c_int64)
        _proto(lib, "sw_radix_sort_u32", c_int32, P, P, P, c_int64, c_int32, P, P, P)
        _proto(lib, "sw_seg_index_scratch_words", c_int64, c_int64, c_int64)
        _proto(lib, "sw_seg_index_max_bytes", c_int64, c_int64)
        _proto(lib, "sw_seg_index", c_int32, P, P, P, P, P, c_int64, P, c_int64, P, P, c_int64, P, c_int64, P, P,
               c_int64, P, P)
        _proto(lib, "sw_seg_index_stamp_words", c_int64, c_int64)
        _proto(lib, "sw_ff_add", c_int32, P, c_int64, c_int64, c_int64, P, P, c_int64, P)
        _proto(lib, "sw_ff_clear", c_int32, P, c_int64, c_int64, c_int64, P)
        _proto(lib, "sw_reject_refs", c_int32, P, P, P, c_int64, P, P, c_int64, P, c_int64, P)
        _proto(lib, "sw_step_snapshot", c_int32, P, P, P, P, c_int32, P, P)
        _proto(lib, "sw_reject_pack", c_int32, P, P, P, P, c_int64, P, P, P)
        _proto(lib, "sw_stream_wait_event", c_int32, P, P)
        _proto(lib, "sw_event_record", c_int32, P, P)
        _proto(lib, "sw_memcpy_h2d_async", c_int32, P, P, c_int64, P)
        _proto(lib, "sw_memset_async", c_int32, P, c_int32, c_int64, P)
        _gpu = lib
        return lib


# launch calls that only enqueue work (microseconds): bound through PyDLL, they keep the GIL
_GPU_BLOCKING = {"sw_sdma_wait"}
_gpu_gil = None


class _GilBound:
    """The kernel library with its enqueue-only entry points bound through ``ctypes.PyDLL`` (the GIL
    stays held: no release / re-acquire per launch) and the blocking ones (``sw_sdma_wait``) through
    ``CDLL``.  A CDLL call gives the GIL up and must win it back from the tenant's busy Python
    threads (store, router, consumers): with the interpreter's 5 ms switch interval an engine step's
    ~20 launches measured ~4 ms of GIL waits per 1M-payload step on a live tenant (profiles/r6_soak)."""

    def __init__(self, cdll):
        self._c = cdll
        self._p = ctypes.PyDLL(cdll._name)

    def __getattr__(self, name):
        f = getattr(self._c, name)
        if name in _GPU_BLOCKING or name.startswith("_"):
            return f
        g = getattr(self._p, name)
        g.restype, g.argtypes = f.restype, f.argtypes
        setattr(self, name, g)
        return g


def gpu_gil():
    """:func:`gpu` with enqueue-only calls keeping the GIL (see :class:`_GilBound`)."""
    global _gpu_gil
    if _gpu_gil is None:
        lib = gpu()
        with _lock:
            if _gpu_gil is None:
                _gpu_gil = _GilBound(lib)
    return _gpu_gil


def gpu_library_path() -> Path:
    return LIB_DIR / "libswgpu.so"

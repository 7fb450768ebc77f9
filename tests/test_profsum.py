"""bench/profsum.py on synthetic rocprofv3 CSVs: kernel classes, idle-gap bins and the attribution
of GPU idle gaps to the host's roctx ranges."""
import csv

from financial_chatbot_llm_amd.bench import profsum


def _write(path, header, rows):
    with open(path, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(header)
        w.writerows(rows)


def _trace(tmp_path):
    # kernels (ns): busy 0-10us, gap 1ms, 1010-1020us, gap 3us, 1023-1030us, gap 2ms, 3030-3040us
    rows = [("gemm_prefill_kernel<1>", 0, 10_000), ("decode_lean_kernel<128>", 1_010_000, 1_020_000),
            ("rmsnorm_kernel<1>", 1_023_000, 1_030_000), ("elementwise_kernel", 3_030_000, 3_040_000)]
    p = tmp_path / "trace.csv"
    _write(p, ["Kernel_Name", "Start_Timestamp", "End_Timestamp"], rows)
    return str(p)


def test_gaps_bins_and_pairs(tmp_path):
    text = profsum.gaps(_trace(tmp_path))
    assert "| 2-5 us | 1 |" in text
    assert "| 0.1-1 ms | 0 |" in text and "| > 1 ms | 2 |" in text   # 1.0 ms and 2.0 ms
    assert "gemm-prefill tile (HIP) -> attention-decode" in text


def test_gaps_by_marker_attributes_to_innermost_engine_range(tmp_path):
    trace = _trace(tmp_path)
    m = tmp_path / "markers.csv"
    # engine thread 7: a step containing a schedule phase over the first gap, a wait over the second;
    # thread 9 (serving loop) encodes a prompt during the second gap
    _write(m, ["Function", "Thread_Id", "Start_Timestamp", "End_Timestamp"], [
        ("engine.step", 7, 0, 4_000_000), ("engine.schedule", 7, 12_000, 1_005_000),
        ("engine.wait", 7, 1_035_000, 3_025_000), ("decode.graph[64]", 7, 3_026_000, 3_028_000),
        ("serve.encode", 9, 1_500_000, 2_500_000)])
    text = profsum.gaps_by_marker(trace, str(m), min_us=100)
    assert "GPU idle gaps >= 100 us: 2," in text
    assert "| engine.schedule | 1 | 0.001 |" in text
    assert "| engine.wait | 1 | 0.002 |" in text
    assert "| engine.wait | serve.encode | 1 |" in text
    assert "| engine.schedule | - | 1 |" in text

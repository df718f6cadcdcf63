"""The ISA checkers and the trace breakdown on synthetic inputs: each must flag the hazard it exists for and pass the
correct form (tools/isa_check.py, tools/glds_wait_audit.py, tools/step_breakdown.py)."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tool(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "tools", f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _gemm_prologue(path, n_after: int, wait: int):
    """A gemm_4w_kernel<10, 0, 224, false> prologue: 15 LDS-DMA ops of K-tile 0, ``n_after`` vector-memory ops after
    them, then ``s_waitcnt vmcnt(wait)`` and the barrier."""
    lines = ["_Z14gemm_4w_kernelILi10ELi0ELi224ELb0EEv8GemmArgs:"]
    lines += ["\tglobal_load_lds_dwordx4 v[2:3], off"] * 15
    lines += ["\tglobal_load_lds_dwordx4 v[4:5], off"] * n_after
    lines += [f"\ts_waitcnt vmcnt({wait})", "\ts_barrier", "\tds_read_b128 v[8:11], v1", "\ts_endpgm",
              ".Lfunc_end0:"]
    path.write_text("\n".join(lines) + "\n")
    return str(path)


@pytest.mark.parametrize("n_after,wait,bad", [(15, 15, 0), (8, 8, 0), (15, 16, 1), (7, 8, 1)])
def test_glds_wait_audit(tmp_path, n_after, wait, bad):
    audit = _tool("glds_wait_audit").audit
    assert audit(_gemm_prologue(tmp_path / "g.s", n_after, wait)) == bad


def test_isa_check_register_hazard(tmp_path):
    isa = _tool("isa_check")
    ok = ["f:", "\tglobal_load_dwordx4 v[4:7], v[0:1], off", "\ts_waitcnt vmcnt(0)", "\tv_add_f32 v8, v4, v5",
          "\ts_endpgm", ".Lfunc_end0:"]
    bad = ["f:", "\tglobal_load_dwordx4 v[4:7], v[0:1], off", "\tv_add_f32 v8, v4, v5", "\ts_waitcnt vmcnt(0)",
           "\ts_endpgm", ".Lfunc_end0:"]
    out = {}
    for name, body in (("ok", ok), ("bad", bad)):
        p = tmp_path / f"{name}.s"
        p.write_text("\n".join(body) + "\n")
        out[name] = [isa.check_function(items) for items in isa.parse_functions(str(p), None).values()]
    assert out["ok"] == [[]] and len(out["bad"][0]) == 1


def test_step_breakdown(tmp_path):
    sb = _tool("step_breakdown")
    hdr = '"Kind","Kernel_Name","Start_Timestamp","End_Timestamp"\n'
    rows, t = [], 0
    for mb in range(4):                     # per micro-batch: a GEMM of 100 ns, a norm of 20 ns, the LSE head of 50
        for name, d in (("gemm_4w_kernel<13, 0, 256, true>(GemmArgs)", 100), ("rmsnorm_f32_kernel<2>(x)", 20),
                        ("gemm_4w_kernel<15, 0, 256, true>(GemmArgs)", 50)):
            rows.append(f'"KERNEL_DISPATCH","{name}",{t},{t + d}\n')
            t += d + 5
    p = tmp_path / "trace.csv"
    p.write_text(hdr + "".join(rows))
    per, calls, tot, span = sb.breakdown(str(p), 2)
    assert per["gemm_4w_kernel<13, 0, 256, true>"] == pytest.approx(0.1)        # us per micro-batch
    assert calls["rmsnorm_f32_kernel<2>"] == 2 and tot == pytest.approx(0.17) and span == pytest.approx(0.185)

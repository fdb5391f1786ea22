"""scripts/isa_audit.py pattern detection on hand-written gfx950 ISA snippets
(no hipcc needed): the serial-stall patterns the round-6 attention / stem /
LayerNorm fixes removed (docs/architecture.md, "Three more ways hipcc
serialises a kernel")."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_spec = importlib.util.spec_from_file_location("isa_audit", os.path.join(ROOT, "scripts", "isa_audit.py"))
isa_audit = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(isa_audit)


def _lines(text):
    return [ln for ln in text.strip("\n").splitlines()]


def test_guarded_load_waited_in_its_branch_is_flagged():
    body = _lines("""
	s_and_saveexec_b64 s[2:3], vcc
	s_cbranch_execz .LBB0_2
	global_load_dwordx4 v[30:33], v55, s[6:7]
	s_waitcnt vmcnt(0)
	global_store_dwordx4 v[2:3], v[30:33], off
.LBB0_2:
	s_or_b64 exec, exec, s[2:3]
	s_endpgm
""")
    assert isa_audit.audit(body)["wait-before-store"] == 1


def test_unconditional_prefetch_is_clean():
    body = _lines("""
	buffer_load_dwordx4 v[0:3], v1, s[4:7], 0 offen
	buffer_load_dwordx4 v[4:7], v1, s[4:7], 0 offen offset:16
	s_waitcnt vmcnt(0)
	buffer_store_dwordx4 v[0:3], v2, s[8:11], 0 offen
	s_endpgm
""")
    r = isa_audit.audit(body)
    assert r["wait-before-store"] == 0 and r["vmcnt0-in-loop"] == 0


def test_lone_lds_read_before_mfma_and_loop_drain_are_flagged():
    body = _lines("""
.LBB1_1:
	ds_read_b128 v[10:13], v5
	s_waitcnt lgkmcnt(0)
	v_mfma_f32_16x16x32_bf16 v[0:3], v[20:23], v[10:13], v[0:3]
	ds_read_b128 v[10:13], v5 offset:64
	ds_read_b128 v[14:17], v5 offset:128
	s_waitcnt lgkmcnt(0)
	v_mfma_f32_16x16x32_bf16 v[0:3], v[20:23], v[10:13], v[0:3]
	s_waitcnt vmcnt(0)
	s_cbranch_scc1 .LBB1_1
	s_endpgm
""")
    r = isa_audit.audit(body)
    assert r["lds-serial"] == 1          # the second wait covers two reads in flight
    assert r["vmcnt0-in-loop"] == 1


def test_integer_bf16_rounding_is_flagged():
    body = _lines("""
	v_bfe_u32 v40, v39, 16, 1
	s_movk_i32 s3, 0x7fff
	v_add3_u32 v40, v39, v40, s3
	v_cvt_pk_bf16_f32 v1, v2, v3
	s_endpgm
""")
    assert isa_audit.audit(body)["int-bf16"] == 1


def test_kernel_bodies_split_on_symbols():
    asm = "\n".join([
        "_Z3fooPf:",
        "\ts_waitcnt vmcnt(0)",
        "\ts_endpgm",
        "_Z3barPf:",
        "\ts_endpgm",
    ])
    names = [sym for sym, _ in isa_audit.kernels(asm)]
    assert names == ["_Z3fooPf", "_Z3barPf"]

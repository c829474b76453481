"""The gfx950 store-data hazard, guarded mechanically (CPU only).

A dwordx3/x4 store reads its data VGPRs after it issues; a VALU write of them with fewer than two wait
states in between changes what is stored (round 4: ~450 wrong sampled picks in 10.5 M until `s_nop 1`
was placed after the record stores). scripts/isa_hazard.py disassembles every gfx950 code object of the
built library and checks the rule over every kernel. This file checks the product library is clean, that
the scan finds the hazard in a scratch build of the decode kernel without the hand-placed wait states,
and the rule itself on small listings."""
import os
import shutil
import subprocess

import pytest

from scripts import isa_hazard as H

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, 'nes-img-captioning_amd', 'nicnes', 'libnicnes.so')
HIPCC = '/opt/rocm/bin/hipcc'
needs_tools = pytest.mark.skipif(not os.path.exists(os.path.join(H.LLVM, 'llvm-objdump')), reason='no ROCm llvm tools')


def _listing(*insns):
    return '0000000000001000 <k>:\n' + ''.join('\t%s // 000000001000: 00000000\n' % i for i in insns)


def test_rule_flags_a_write_right_behind_the_store():
    asm = _listing('buffer_store_dwordx4 v[108:111], v0, s[48:51], s0 offen nt', 'v_mov_b64_e32 v[108:109], 0')
    assert H.scan(asm) == [('k', 'buffer_store_dwordx4 v[108:111], v0, s[48:51], s0 offen nt',
                            'v_mov_b64_e32 v[108:109], 0', 0)]


def test_rule_counts_wait_states():
    st = 'global_store_dwordx4 v[2:3], v[8:11], off'
    assert H.scan(_listing(st, 's_nop 1', 'v_mov_b32_e32 v9, 0')) == []          # 2 wait states
    assert len(H.scan(_listing(st, 's_nop 0', 'v_mov_b32_e32 v9, 0'))) == 1      # 1 is not enough
    assert len(H.scan(_listing(st, 's_add_u32 s0, s0, 4', 'v_add_f32_e32 v11, v1, v2'))) == 1
    assert H.scan(_listing(st, 's_add_u32 s0, s0, 4', 's_mov_b32 s1, 0', 'v_mov_b32_e32 v9, 0')) == []
    assert H.scan(_listing(st, 'v_mov_b32_e32 v2, 0')) == []                    # the address, not the data
    assert H.scan(_listing('buffer_store_dwordx2 v[8:9], v0, s[0:3], 0 offen', 'v_mov_b32_e32 v8, 0')) == []
    assert len(H.scan(_listing('scratch_store_dwordx3 off, v[4:6], s33', 's_cbranch_scc1 4',
                               'v_mov_b32_e32 v6, 1'))) == 1                    # fall-through path
    assert H.scan(_listing(st, 's_branch 8', 'v_mov_b32_e32 v9, 0')) == []


@needs_tools
def test_product_library_has_no_store_data_hazard():
    if not os.path.exists(LIB):
        pytest.fail('libnicnes.so not built (make -C nes-img-captioning_amd)')
    counts = {}
    hits = H.scan_library(LIB, counts)
    assert counts['code_objects'] == 5                      # decode, cider, update, sensitivity, engine
    assert counts['wide_stores'] >= 50                      # the scan sees the kernels' 16-byte stores
    assert hits == [], '\n'.join('%s: %s -> %s (%d wait states)' % h for h in hits)


@needs_tools
@pytest.mark.skipif(not os.path.exists(HIPCC), reason='no hipcc')
def test_scan_catches_the_build_without_the_wait_states(tmp_path):
    """The decode kernel compiled without the hand-placed `s_nop 1` (NICNES_STORE_WAITS=0, a scratch build
    never linked into the product) shows the round-4 pattern: the block sum zeroed right behind its store."""
    src = os.path.join(REPO, 'nes-img-captioning_amd', 'csrc', 'decode_kernel.hip')
    obj = str(tmp_path / 'decode_nowait.o')
    subprocess.check_call([HIPCC, '--offload-arch=gfx950', '-O3', '-std=c++17', '-ffp-contract=off', '-fPIC',
                           '-DNICNES_STORE_WAITS=0', '-x', 'hip', '-c', src, '-o', obj])
    hits = H.scan_library(obj)
    assert hits, 'the scan no longer sees the hazard it guards against'
    assert all('nicnes_decode_steps_kernelILb0ELb1E' in fn for fn, _, _, _ in hits)   # the sampled instantiation
    assert all(w < H.MIN_WAIT_STATES for _, _, _, w in hits)

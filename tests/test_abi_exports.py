"""The C-ABI library loads and exports every function include/*.h declares (no GPU calls)."""
import ctypes as C
import os
import re

import pytest

from conftest import ROOT


def declared(header):
    txt = open(os.path.join(ROOT, 'include', header)).read()
    txt = re.sub(r'/\*.*?\*/', '', txt, flags=re.S)
    return sorted(set(re.findall(r'\b(avr_[a-z0-9_]+)\s*\(', txt)))


def test_header_declares_the_boundary():
    names = declared('avr.h')
    for must in ('avr_create', 'avr_destroy', 'avr_reset', 'avr_step', 'avr_step_device', 'avr_set_state', 'avr_get_state',
                 'avr_last_error'):
        assert must in names


def test_libavr_exports_every_declared_symbol(libavr_path):
    lib = C.CDLL(libavr_path)
    missing = [n for n in declared('avr.h') if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_list_matches_header():
    from avr import _lib
    assert set(_lib.EXPORTS) <= set(declared('avr.h'))
    assert set(declared('avr.h')) - set(_lib.EXPORTS) <= {'avr_set_profile_buffer'}


def test_abi_constants(libavr_path):
    lib = C.CDLL(libavr_path)
    from avr import _abi as ABI
    lib.avr_state_words.restype = C.c_int32
    assert lib.avr_state_words() == ABI.STATE_WORDS
    lib.avr_abi_version.restype = C.c_int32
    assert lib.avr_abi_version() >= 1


def test_model_desc_struct_matches_header():
    """ctypes mirror of avr_model_desc: every field of include/avr_model.h is present."""
    from avr import _abi as ABI
    txt = open(os.path.join(ROOT, 'include', 'avr_model.h')).read()
    body = txt[txt.index('typedef struct avr_model_desc'):]
    body = body[:body.index('} avr_model_desc;')]
    body = re.sub(r'/\*.*?\*/', '', body, flags=re.S)
    body = body[body.index('{') + 1:]
    fields = []
    for stmt in body.split(';'):
        stmt = re.sub(r'^\s*(const\s+)?(u?int\d+_t|double|float|char)\s*', '', stmt.strip())
        for decl in stmt.split(','):
            decl = re.sub(r'\[[^\]]*\]', '', decl).replace('*', '').strip()
            if decl:
                fields.append(decl)
    mirror = [f[0] for f in ABI.avr_model_desc._fields_]
    assert fields == mirror


def test_oracle_exports(oracle_built):
    from oracle import oracle
    lib = oracle.lib('f64')
    for n in ('avr_oracle_create', 'avr_oracle_step', 'avr_oracle_settle', 'avr_oracle_substep', 'avr_oracle_narrowphase',
              'avr_oracle_robot_fk', 'avr_oracle_set_threads'):
        assert hasattr(lib, n)

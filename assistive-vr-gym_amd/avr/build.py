"""In-tree build of the native artefacts: libavr.so (hipcc, gfx950) and the CPU oracle (gcc).

`python -m avr.build` or `__graft_entry__.build()`.  No torch extension machinery: the product
is a plain C-ABI shared library loaded with ctypes.
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, 'csrc')
LIB = os.path.join(HERE, 'libavr.so')
ARCH = os.environ.get('AVR_OFFLOAD_ARCH', 'gfx950')
# one translation unit per task (the shared kernel / C-ABI sources instantiated in a namespace,
# csrc/avr_task_tu.h), the extern "C" dispatcher, the hull support tables
SOURCES = ['avr_task_feeding.hip', 'avr_task_scratch.hip', 'avr_task_bedbath.hip', 'avr_dressing.hip', 'avr_api.cpp', 'avr_hulltab.cpp']
HEADERS = ['avr_math.h', 'avr_kmodel.h', 'avr_task.h', 'avr_task_tu.h', 'avr_kernel.hip', 'avr_capi.hip', 'avr_glue_scratch.hip', 'avr_glue_bedbath.hip', 'avr_reset_ik.hip', 'avr_base_search.hip']
OBJDIR = os.path.join(PKG, 'build')


def _hipcc():
    for c in (os.environ.get('HIPCC'), '/opt/rocm/bin/hipcc', shutil.which('hipcc')):
        if c and os.path.exists(c):
            return c
    raise RuntimeError('hipcc not found')


_COMPILER_ID = {}


def _compiler_id(cc):
    """The compiler's own version banner (first two lines of `<cc> --version`): recorded beside the
    command line, so a library built by another hipcc / clang release is rebuilt from source."""
    if cc not in _COMPILER_ID:
        try:
            out = subprocess.run([cc, '--version'], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True).stdout
        except OSError:
            out = ''
        _COMPILER_ID[cc] = ' | '.join(out.strip().splitlines()[:2])
    return _COMPILER_ID[cc]


def _stamp(cmd):
    return ' '.join(cmd) + '\n# compiler: ' + _compiler_id(cmd[0])


def _stale(target, deps, cmd):
    """Rebuild when the target is missing, older than a dependency, or was built by a different
    command line or compiler release (recorded in <target>.cmd: flags, sources and the compiler's
    version banner, so a flag change or another toolchain rebuilds)."""
    if not os.path.exists(target):
        return True
    side = target + '.cmd'
    if not os.path.exists(side) or open(side).read() != _stamp(cmd):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


_PROBED = {}
_PROBE_CACHE = os.path.join(HERE, '.hipcc_probe')     # probe results survive across processes


def _supported(flags):
    """True if hipcc accepts `flags` (probed once per flag set on an empty gfx950 kernel; the result
    is cached on disk next to the library, keyed by the hipcc path and the flags)."""
    key = tuple(flags)
    ckey = '%s %s' % (_hipcc(), ' '.join(flags))
    if key not in _PROBED and os.path.exists(_PROBE_CACHE):
        for line in open(_PROBE_CACHE):
            k, _, v = line.rstrip('\n').rpartition('\t')
            if k == ckey:
                _PROBED[key] = v == '1'
    if key not in _PROBED:
        import tempfile
        with tempfile.TemporaryDirectory() as d:
            src = os.path.join(d, 'p.hip')
            open(src, 'w').write('__global__ void k() {}\n')
            r = subprocess.run([_hipcc(), '--offload-arch=%s' % ARCH, '--cuda-device-only', '-c', '-o', os.path.join(d, 'p.o'), src] + list(flags),
                               stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            _PROBED[key] = r.returncode == 0
        with open(_PROBE_CACHE, 'a') as f:
            f.write('%s\t%d\n' % (ckey, int(_PROBED[key])))
    return _PROBED[key]


# AMDGPU register-pressure trackers in the scheduler: part B 0.590 -> 0.564 ms, A 0.552 -> 0.560 ms,
# 356k -> 361k env-steps/s (round 1 flag sweep; tools/build_variants.py + tools/gpu_variants.sh
# rerun such sweeps).  An internal LLVM option: dropped (with a warning) when this hipcc does not
# know it.
TRACKERS = ('-mllvm', '-amdgpu-use-amdgpu-trackers=1')


def lib_flags(extra=()):
    flags = ['--offload-arch=%s' % ARCH, '-O3', '-std=c++17', '-fPIC', '-Wno-unused-result', '-fno-slp-vectorize']
    if _supported(TRACKERS):
        flags += list(TRACKERS)
    else:
        sys.stderr.write('avr.build: hipcc does not accept %s; building without it\n' % ' '.join(TRACKERS))
    return flags + list(extra)


def lib_cmd(extra=(), out=LIB):
    """The full build as one command line (recorded in <lib>.cmd: a flag change rebuilds)."""
    return [_hipcc()] + lib_flags(extra) + ['-shared', '-o', out] + [os.path.join(CSRC, f) for f in SOURCES]


def build_lib(force=False, extra=(), out=LIB):
    """Compile the translation units in parallel (one hipcc per TU), then link libavr*.so."""
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, 'include', h) for h in ('avr.h', 'avr_model.h', 'avr_dressing.h')] + [os.path.abspath(__file__)]
    cmd = lib_cmd(extra, out)
    if not force and not _stale(out, deps, cmd):
        return out
    tag = os.path.splitext(os.path.basename(out))[0]
    os.makedirs(OBJDIR, exist_ok=True)
    flags = lib_flags(extra)
    procs, objs = [], []
    for f in SOURCES:
        o = os.path.join(OBJDIR, '%s.%s.o' % (tag, os.path.splitext(f)[0]))
        objs.append(o)
        procs.append(subprocess.Popen([_hipcc()] + flags + ['-c', '-o', o, os.path.join(CSRC, f)]))
    if any(p.wait() != 0 for p in procs):
        raise subprocess.CalledProcessError(1, 'hipcc (%s)' % out)
    subprocess.check_call([_hipcc(), '--offload-arch=%s' % ARCH, '-shared', '-fPIC', '-o', out] + objs)
    open(out + '.cmd', 'w').write(_stamp(cmd))
    return out


def build_prof(force=False):
    """Diagnostic build with per-phase s_memtime counters (tools/prof_phases.py); never shipped."""
    return build_lib(force=force, extra=('-DAVR_PROF',), out=os.path.join(HERE, 'libavr_prof.so'))


def build_poison(force=False):
    """Diagnostic build whose kernels NaN-fill their LDS blocks at entry (-DAVR_LDS_POISON): any
    read of an LDS word the kernel did not write this launch changes its results
    (tests/test_gpu_parity.py::test_lds_poison_build_is_bit_identical); never shipped."""
    return build_lib(force=force, extra=('-DAVR_LDS_POISON',), out=os.path.join(HERE, 'libavr_poison.so'))


def build_wavetime(force=False):
    """Diagnostic build with per-wave start/end stamps (tools/wavetime.py); never shipped."""
    return build_lib(force=force, extra=('-DAVR_WAVETIME',), out=os.path.join(HERE, 'libavr_wt.so'))


def header_defines(path, prefix):
    """Numeric #defines NAME -> value of a C header (the constants shared with the kernels)."""
    import re
    env = {}
    for line in open(path):
        m = re.match(r'#define\s+(%s\w+)\s+(.+?)\s*(/\*.*)?$' % prefix, line)
        if not m:
            continue
        expr = m.group(2)
        for k in sorted(env, key=len, reverse=True):
            expr = expr.replace(k, repr(env[k]))
        try:
            env[m.group(1)] = eval(expr, {'__builtins__': {}})
        except Exception:
            pass
    return env


DRESSING_HEADER = os.path.join(ROOT, 'include', 'avr_dressing.h')
DRESSING_CONSTS = os.path.join(HERE, '_dressing_consts.py')


def dressing_consts_source():
    d = header_defines(DRESSING_HEADER, 'AVR_DR_')
    lines = ['"""DressingJaco-v0 constants (include/avr_dressing.h), generated by avr.build.write_dressing_consts();',
             'tests/test_dressing.py checks them against the header.  Do not edit by hand."""', '', 'DEFINES = {']
    lines += ['    %r: %r,' % (k, v) for k, v in d.items()]
    return '\n'.join(lines + ['}']) + '\n'


def write_dressing_consts():
    """Regenerate avr/_dressing_consts.py from include/avr_dressing.h when they differ."""
    src = dressing_consts_source()
    if not os.path.exists(DRESSING_CONSTS) or open(DRESSING_CONSTS).read() != src:
        open(DRESSING_CONSTS, 'w').write(src)


def build_oracle():
    subprocess.check_call(['make', '-s', '-C', os.path.join(ROOT, 'oracle')])


def build_all(force=False):
    write_dressing_consts()
    build_lib(force=force)
    build_poison(force=force)
    build_oracle()


if __name__ == '__main__':
    build_all(force='--force' in sys.argv)
    if '--prof' in sys.argv:
        build_prof(force=True)
    if '--wt' in sys.argv:
        build_wavetime(force=True)
    print(LIB)

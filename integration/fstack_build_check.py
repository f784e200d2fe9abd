#!/usr/bin/env python3
"""Compile F-Stack's kernel domain with IPsec and the MI355X driver, and check
that the relocatable object F-Stack links from it has no unresolved symbol.

    python integration/fstack_build_check.py [--ref /root/reference] [--work DIR]

What it does ("Proving the build"):

1. Copies the F-Stack files it needs (lib/, mk/; freebsd/ by symlink) into
   WORK, and applies integration/apply_fstack.sh (the patch plus
   ff_gpucrypto.c, ff_gpucrypto_host.c and ff_newbus.c into lib/).
2. Drops lib/Makefile's `pkg-config --exists libdpdk` guard in the copy: DPDK
   is not installed here and the kernel domain does not use it (its flags feed
   only HOST_CFLAGS).  Everything else is lib/Makefile's own: the generated
   headers (machine_includes, *_if.h / *_if.c from the .m files, vnode_if.h,
   filtered_predefined_macros.h) and every kernel-domain object (`OBJS`) of a
   `FF_IPSEC=1 FF_IPSEC_GPU=1` build, compiled with its NORMAL_C rule
   (-nostdinc, FreeBSD headers, -Werror).
3. `ld -d -r` of all those objects, as the libfstack.a rule does first, then
   every undefined symbol of the result must be one of:
     - linker-generated (__start_set_* / __stop_set_* linker sets, _DYNAMIC,
       _GLOBAL_OFFSET_TABLE_);
     - defined by a host-domain source (FF_HOST_SRCS): compiled here with
       HOST_CFLAGS where its headers exist, otherwise (DPDK headers) read from
       the source text's top-level definitions, and the blocking header named;
     - exported by the C library the application links (libc.so.6).
   and the kernel-domain entry points the host shim calls must be defined and
   listed in lib/ff_api.symlist (they survive the localize step).

Prints a JSON report; exit status 0 only when nothing is unresolved.
"""
import argparse
import json
import os
import re
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
MAKEVARS = r"""
print-objs:
	@echo $(OBJS)
print-host-srcs:
	@echo $(HOST_SRCS)
print-host-c:
	@echo $(CC) -c $(HOST_CFLAGS) $(HOST_INCLUDES)
kgen: machine_includes $(MHEADERS) $(MSRCS) $(IMACROS_FILE)
kobjs: $(OBJS)
"""
LINKER = re.compile(r"^(__(start|stop)_set_\w+|_DYNAMIC|_GLOBAL_OFFSET_TABLE_)$")


def run(cmd, cwd=None, check=True):
    r = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True, shell=isinstance(cmd, str))
    if check and r.returncode != 0:
        raise RuntimeError(f"{cmd}: rc {r.returncode}\n{r.stdout[-4000:]}\n{r.stderr[-4000:]}")
    return r


def nm_defined(path, dynamic=False):
    flags = ["-D"] if dynamic else []
    out = run(["nm", "--defined-only"] + flags + [path]).stdout
    return {l.split()[-1].split("@")[0] for l in out.splitlines() if len(l.split()) >= 2}


def body_follows(lines, k):
    """Whether the parenthesised list opened on line k is followed by a
    function body (a definition) rather than ';' (a prototype)."""
    rest = "\n".join(lines[k:k + 40])
    depth = 0
    for i, ch in enumerate(rest):
        depth += ch == "("
        depth -= ch == ")"
        if ch == ")" and depth == 0:
            tail = re.sub(r"__attribute__\s*\(\(.*?\)\)", "", rest[i + 1:i + 200], flags=re.S)
            return tail.lstrip().startswith("{")
    return False


def c_definitions(text):
    """External (non-static) functions and variables defined at file scope of
    a C source, read from its text (the host files whose DPDK headers are
    absent): F-Stack writes file-scope definitions from column 0, the
    function name either at column 0 under its return type (BSD style) or
    after it on the same line."""
    text = re.sub(r"/\*.*?\*/", lambda m: "\n" * m.group(0).count("\n"), text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    lines = text.split("\n")
    names = set()
    kw = ("static", "extern", "typedef", "return", "if", "else", "for", "while", "switch", "case")
    for k, l in enumerate(lines):
        if not l or l[0] in " \t#}{":
            continue
        prev = ""
        for p in range(k - 1, -1, -1):
            if lines[p].strip():
                prev = lines[p]
                break
        m = re.match(r"(\w+)\s*\(", l)
        if m and m.group(1) not in kw:
            if prev and prev[0] not in " \t#}{" and not re.search(r"[;,)]\s*$", prev) \
                    and not re.match(r"(static|extern|typedef)\b", prev) and body_follows(lines, k):
                names.add(m.group(1))                       # BSD style: type on the line above
            continue
        if re.match(r"(static|extern|typedef)\b", l):
            continue
        m = re.match(r"(?:const\s+)?(?:unsigned\s+|signed\s+|struct\s+\w+\s+|enum\s+\w+\s+|union\s+\w+\s+)?"
                     r"\w+[\s\*]+(\w+)\s*\(", l)
        if m and not l.rstrip().endswith(";"):
            names.add(m.group(1))                           # one-line function head
            continue
        m = re.match(r"(?:const\s+)?(?:struct\s+\w+|enum\s+\w+|union\s+\w+|unsigned\s+\w+|\w+)[\s\*]+"
                     r"(\w+)\s*(\[[^\]]*\])*\s*(=|;)", l)
        if m:
            names.add(m.group(1))                           # variable definition
    return names


def build_kernel(ref, work, jobs, extra_make=""):
    """Copy + patch the F-Stack tree into `work` and compile every kernel-domain
    object with lib/Makefile's own rules.  -> (lib dir, make argv, objects,
    report, make's return code)"""
    if os.path.isdir(work):
        shutil.rmtree(work)
    os.makedirs(work)
    for d in ("lib", "mk"):
        shutil.copytree(os.path.join(ref, d), os.path.join(work, d), symlinks=True)
    os.symlink(os.path.join(ref, "freebsd"), os.path.join(work, "freebsd"))
    run(["sh", os.path.join(HERE, "apply_fstack.sh"), work])
    lib = os.path.join(work, "lib")
    mk = os.path.join(lib, "Makefile")
    text = open(mk).read()
    guard = re.search(r"ifneq \(\$\(shell pkg-config --exists libdpdk && echo 0\),0\)\n.*\nendif\n", text)
    assert guard, "lib/Makefile's DPDK guard not found"
    open(mk, "w").write(text.replace(guard.group(0), "# (DPDK guard dropped: kernel-domain check)\n"))
    open(os.path.join(work, "vars.mk"), "w").write(MAKEVARS + extra_make)
    make = ["make", "-s", "-f", "Makefile", "-f", "../vars.mk", "FF_IPSEC=1", "FF_IPSEC_GPU=1",
            "ESPGPU_ROOT=" + os.path.dirname(HERE)]
    run(make + ["kgen"], cwd=lib)
    r = run(make + ["-k", f"-j{jobs}", "kobjs"], cwd=lib, check=False)
    errors = [l for l in (r.stdout + r.stderr).splitlines() if "error" in l]
    objs = run(make + ["print-objs"], cwd=lib).stdout.split()
    report = {"kernel_objects": len(objs), "compile_errors": errors}
    return lib, make, objs, report, r.returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--work", default="/tmp/fstack_build_check")
    ap.add_argument("-j", type=int, default=8)
    a = ap.parse_args()
    lib, make, objs, report, rc = build_kernel(a.ref, a.work, a.j)
    errors = report["compile_errors"]
    if rc != 0:
        report["unresolved"] = ["<kernel-domain compile failed>"]
        print(json.dumps(report, indent=1))
        return 1
    ro = os.path.join(a.work, "libfstack.ro")
    run(["ld", "-d", "-r", "-o", ro] + objs, cwd=lib)
    undef = sorted({l.split()[-1] for l in run(["nm", "-u", ro]).stdout.splitlines()})
    kdef = nm_defined(ro)

    # host domain: compile what builds without DPDK, read the rest
    host_c = run(make + ["print-host-c"], cwd=lib).stdout.split()
    host_def, compiled, blocked = set(), [], {}
    for src in run(make + ["print-host-srcs"], cwd=lib).stdout.split():
        obj = os.path.join(a.work, src.replace(".c", ".host.o"))
        rr = run(host_c + [src, "-o", obj], cwd=lib, check=False)
        if rr.returncode == 0:
            host_def |= nm_defined(obj)
            compiled.append(src)
            continue
        m = re.search(r"fatal error: ([\w./-]+): No such file", rr.stderr)
        first = next((l for l in rr.stderr.splitlines() if "error:" in l), rr.stderr.strip()[-200:])
        blocked[src] = m.group(1) if m else first[:200]
        host_def |= c_definitions(open(os.path.join(lib, src), errors="replace").read())
    libc = run(["gcc", "-print-file-name=libc.so.6"]).stdout.strip()
    if not os.path.isabs(libc):
        libc = next(p for p in ("/lib/x86_64-linux-gnu/libc.so.6", "/lib64/libc.so.6",
                                "/usr/lib64/libc.so.6") if os.path.exists(p))
    libc_def = nm_defined(os.path.realpath(libc), dynamic=True)

    where = {"linker": [], "host": [], "libc": []}
    unresolved = []
    for s in undef:
        if LINKER.match(s):
            where["linker"].append(s)
        elif s in host_def:
            where["host"].append(s)
        elif s in libc_def:
            where["libc"].append(s)
        else:
            unresolved.append(s)
    symlist = set(open(os.path.join(lib, "ff_api.symlist")).read().split())
    exports = ["ff_gpucrypto_done", "ff_gpucrypto_unblock"]
    missing_exports = [s for s in exports if s not in kdef or s not in symlist]
    report.update({
        "undefined": len(undef), "resolved_by": {k: len(v) for k, v in where.items()},
        "host_compiled": compiled, "host_blocked": blocked,
        "gpu_driver_calls_host": sorted(s for s in where["host"] if s.startswith("ff_gpucrypto_host")),
        "missing_exports": missing_exports, "unresolved": unresolved,
    })
    print(json.dumps(report, indent=1))
    return 0 if not unresolved and not missing_exports and not errors else 1


if __name__ == "__main__":
    sys.exit(main())

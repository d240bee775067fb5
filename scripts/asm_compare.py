#!/usr/bin/env python3
"""Compare two builds of the HIP sources function by function, at the assembly level.

    python scripts/asm_compare.py DIR_A DIR_B        # dirs of <tu>.dev.s / <tu>.host.s files

Made with `hipcc <the Makefile's flags> --cuda-device-only -S` (and --cuda-host-only) per source
file.  Each function's body (device: kernel code + its .amdhsa_kernel descriptor; host: the x86
text) is normalised for label numbering and compared; prints the functions that differ, exist in
one build only, and a summary.  Used to show that a source clean-up (dead A/B branches removed)
leaves every kept kernel's and host function's code unchanged.
"""
import os
import re
import sys

FUNC = re.compile(r"^([A-Za-z_.$][\w.$]*):\s*(?:;.*|#.*|//.*)?$")


def split(path):
    out, cur, name = {}, [], None
    lines = open(path).read().splitlines()
    for ln in lines:
        m = re.match(r"^\s*\.type\s+([\w.$]+),\s*@function", ln)
        if m:
            name, cur = m.group(1), []
            continue
        if name is not None:
            if re.match(r"^\.Lfunc_end\d+:", ln):
                out[name] = cur
                name = None
                continue
            cur.append(ln)
    # device kernel descriptors
    desc, dname = {}, None
    for ln in lines:
        m = re.match(r"^\s*\.amdhsa_kernel\s+(\S+)", ln)
        if m:
            dname, desc[m.group(1)] = m.group(1), []
            continue
        if dname is not None:
            if ".end_amdhsa_kernel" in ln:
                dname = None
                continue
            desc[dname].append(ln)
    for k, v in desc.items():
        out.setdefault(k, []).extend(["#desc"] + v)
    return out


def norm(body):
    res = []
    for ln in body:
        if not ln.strip().startswith("#desc"):
            ln = re.sub(r"\s+#.*$", "", ln.split(";")[0].split("//")[0]).rstrip()  # device ; / host # comments
            if ln.lstrip().startswith("#"):
                continue
        if not ln.strip() or ln.strip().startswith(("; %bb", ".loc", ".file", ".cfi")):
            continue
        ln = re.sub(r"\.LBB\d+_(\d+)", r".LBB_\1", ln)
        ln = re.sub(r"\.Ltmp\d+", ".Ltmp", ln)
        ln = re.sub(r"\.Lfunc_end\d+", ".Lfunc_end", ln)
        ln = re.sub(r"\.LJTI\d+_(\d+)", r".LJTI_\1", ln)
        ln = re.sub(r"\.LCPI\d+_(\d+)", r".LCPI_\1", ln)
        ln = re.sub(r"\.L\.str(\.\d+)?", ".L.str", ln)
        ln = re.sub(r"__hip_cuid_\w+", "__hip_cuid", ln)
        ln = re.sub(r"__hip_gpubin_handle_\w+", "__hip_gpubin_handle", ln)
        res.append(ln)
    return res


def main(a, b):
    same = diff = only_a = only_b = 0
    for fn in sorted(os.listdir(a)):
        if not fn.endswith(".s"):
            continue
        fa, fb = split(os.path.join(a, fn)), split(os.path.join(b, fn)) if os.path.exists(os.path.join(b, fn)) else {}
        for k in sorted(set(fa) | set(fb)):
            if k not in fb:
                only_a += 1
                print(f"only in A  {fn}: {k}")
            elif k not in fa:
                only_b += 1
                print(f"only in B  {fn}: {k}")
            elif norm(fa[k]) != norm(fb[k]):
                diff += 1
                print(f"DIFFERENT  {fn}: {k}")
            else:
                same += 1
    print(f"identical {same}, different {diff}, only in A {only_a}, only in B {only_b}")
    return 1 if diff else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2]))

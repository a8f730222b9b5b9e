"""Minimal `unifdef`: resolve the preprocessor conditionals of the named macros only.

    python tools/unifdef.py -DFOO -UBAR file.hip > out.hip

Handles `#ifdef X`, `#ifndef X`, `#if defined(X)`, `#elif defined(X)`, `#else`, `#endif` (nested);
conditionals on any other macro are left as they are. Used to keep timing-only ablations and
diagnostic builds out of the product sources: `tools/make_variant_patches.sh` records each one
as a patch under `tools/variants/`, which `tools/build_variant.sh` applies to a copy of the tree.
"""
import re
import sys

DIR = re.compile(r"^\s*#\s*(ifdef|ifndef|if|elif|else|endif)\b\s*(.*)$")
DEFINED = re.compile(r"^(!?)\s*defined\s*\(?\s*(\w+)\s*\)?\s*(//.*)?$")


def resolve(lines, defs, undefs):
    known = defs | undefs
    out = []
    # stack entries: (managed, emitting_now, branch_taken, parent_emitting)
    stack = []
    emitting = True
    for ln in lines:
        m = DIR.match(ln)
        if not m:
            if emitting:
                out.append(ln)
            continue
        kw, rest = m.group(1), m.group(2).strip()
        if kw in ("ifdef", "ifndef", "if"):
            name, neg = None, False
            if kw in ("ifdef", "ifndef"):
                name = rest.split()[0] if rest else None
                neg = kw == "ifndef"
            else:
                d = DEFINED.match(rest)
                if d:
                    neg, name = d.group(1) == "!", d.group(2)
            if name in known:
                val = (name in defs) != neg
                stack.append([True, None, val, emitting])
                emitting = emitting and val
            else:
                stack.append([False, None, None, emitting])
                if emitting:
                    out.append(ln)
            continue
        if not stack:
            raise SystemExit(f"unbalanced #{kw}")
        top = stack[-1]
        managed, _, taken, parent = top
        if kw == "elif":
            d = DEFINED.match(rest)
            if managed:
                if d is None or d.group(2) not in known:
                    raise SystemExit(f"#elif on an unmanaged condition after a managed #if: {ln!r}")
                val = (d.group(2) in defs) != (d.group(1) == "!")
                emitting = parent and (not taken) and val
                top[2] = taken or val
            else:
                if d is not None and d.group(2) in known:
                    raise SystemExit(f"managed #elif inside an unmanaged #if: {ln!r}")
                if parent:
                    out.append(ln)
        elif kw == "else":
            if managed:
                emitting = parent and not taken
                top[2] = True
            elif parent:
                out.append(ln)
        elif kw == "endif":
            stack.pop()
            emitting = parent
            if not managed and parent:
                out.append(ln)
    if stack:
        raise SystemExit("unterminated conditional")
    return out


def main(argv):
    defs, undefs, files = set(), set(), []
    for a in argv:
        if a.startswith("-D"):
            defs.add(a[2:])
        elif a.startswith("-U"):
            undefs.add(a[2:])
        else:
            files.append(a)
    for f in files:
        with open(f) as fh:
            sys.stdout.write("".join(resolve(fh.readlines(), defs, undefs)))


if __name__ == "__main__":
    main(sys.argv[1:])

"""Offline codestyle gate (reference ``codestyle/`` hooks):
line length <= 120, no tabs / trailing whitespace / merge markers, every
Python module has a docstring, every kernel source starts with a comment
header, and Python files compile.

    python tools/codestyle.py [files...]      (default: the whole tree)
"""
import ast
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAXLEN = 120
SKIP_DIRS = {".git", "build", "__pycache__", "gpurun_out", ".pytest_cache"}


def _files(args):
    if args:
        return [a for a in args if a.endswith((".py", ".hip", ".cpp", ".h"))]
    out = []
    for r, ds, fs in os.walk(ROOT):
        ds[:] = [d for d in ds if d not in SKIP_DIRS]
        out += [os.path.join(r, f) for f in fs if f.endswith((".py", ".hip", ".cpp", ".h"))]
    return out


def check(path):
    errs = []
    text = open(path, encoding="utf-8").read()
    for i, line in enumerate(text.splitlines(), 1):
        if len(line) > MAXLEN:
            errs.append("%s:%d: line longer than %d" % (path, i, MAXLEN))
        if "\t" in line and path.endswith(".py"):
            errs.append("%s:%d: tab" % (path, i))
        if line != line.rstrip():
            errs.append("%s:%d: trailing whitespace" % (path, i))
        if line.startswith(("<<<<<<<", ">>>>>>>")):
            errs.append("%s:%d: merge marker" % (path, i))
    if path.endswith(".py"):
        try:
            tree = ast.parse(text, path)
        except SyntaxError as e:
            return errs + ["%s: %s" % (path, e)]
        if text.strip() and not ast.get_docstring(tree) and not path.endswith("__init__.py"):
            errs.append("%s: missing module docstring" % path)
    elif text and not text.lstrip().startswith("//"):
        errs.append("%s: missing header comment" % path)
    return errs


def main(argv=None):
    errs = []
    for f in _files(sys.argv[1:] if argv is None else argv):
        errs += check(f)
    for e in errs:
        print(e)
    return 1 if errs else 0


if __name__ == "__main__":
    sys.exit(main())

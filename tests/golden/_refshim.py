"""In-memory py2->py3 import shim for the p265 reference (fixture generation only).

THIS CONTAINER ONLY. Nothing under tests/ imports this module at test time; it is
used by the committed generator scripts in this directory to run the read-only
Python-2 reference at /root/reference and capture golden vectors from it.  The
reference never travels to the GPU box: only the .npz/.json vectors it produces
are committed.

Recipe: every module under /root/reference/decoder (and
/root/reference/dec.py) is read as text, passed through lib2to3's print fixer,
parsed, has ``/`` rewritten to ``//`` unless an operand contains a ``float(...)``
call (py2 integer division semantics; keeps bsb.py:155 / sps.py:151 true
division), and is exec'd into ONE shared module object per name, whether it is
imported as ``decoder.X`` or as the bare implicit-relative ``X``.  No file is
written under /root/reference (bytecode writing is disabled).
"""
import ast
import importlib.abc
import importlib.machinery
import logging
import os
import sys
import warnings

REF_ROOT = "/root/reference"
REF_DECODER = os.path.join(REF_ROOT, "decoder")

sys.dont_write_bytecode = True
os.environ.setdefault("MPLBACKEND", "Agg")


class _DivToFloorDiv(ast.NodeTransformer):
    @staticmethod
    def _has_float(node):
        for n in ast.walk(node):
            if isinstance(n, ast.Call) and isinstance(n.func, ast.Name) and n.func.id == "float":
                return True
        return False

    def visit_BinOp(self, node):
        self.generic_visit(node)
        if isinstance(node.op, ast.Div) and not (self._has_float(node.left) or self._has_float(node.right)):
            node.op = ast.FloorDiv()
        return node

    def visit_AugAssign(self, node):
        self.generic_visit(node)
        if isinstance(node.op, ast.Div) and not self._has_float(node.value):
            node.op = ast.FloorDiv()
        return node


def _py2_to_py3(src, filename):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        from lib2to3 import refactor
        tool = refactor.RefactoringTool(["lib2to3.fixes.fix_print"])
        src = str(tool.refactor_string(src if src.endswith("\n") else src + "\n", filename))
    tree = _DivToFloorDiv().visit(ast.parse(src, filename))
    ast.fix_missing_locations(tree)
    return compile(tree, filename, "exec")


class _RefLoader(importlib.abc.Loader):
    def __init__(self, path):
        self.path = path

    def create_module(self, spec):
        return None

    def exec_module(self, module):
        with open(self.path) as f:
            code = _py2_to_py3(f.read(), self.path)
        exec(code, module.__dict__)


class _RefFinder(importlib.abc.MetaPathFinder):
    """Maps decoder, decoder.X, bare X (X in decoder/*.py) and dec to one module each."""

    def __init__(self):
        self.names = {os.path.splitext(f)[0] for f in os.listdir(REF_DECODER)
                      if f.endswith(".py") and f != "__init__.py"}

    def find_spec(self, fullname, path=None, target=None):
        if fullname == "decoder":
            spec = importlib.machinery.ModuleSpec(fullname, None, is_package=True)
            spec.submodule_search_locations = [REF_DECODER]
            return spec
        if fullname == "dec":
            return importlib.machinery.ModuleSpec(fullname, _RefLoader(os.path.join(REF_ROOT, "dec.py")))
        short = fullname[len("decoder."):] if fullname.startswith("decoder.") else fullname
        if short in self.names:
            other = ("decoder." + short) if fullname == short else short
            if other in sys.modules:          # alias: one shared module object
                sys.modules[fullname] = sys.modules[other]
                return importlib.machinery.ModuleSpec(fullname, _AliasLoader(sys.modules[other]))
            return importlib.machinery.ModuleSpec(fullname, _RefLoader(os.path.join(REF_DECODER, short + ".py")))
        return None


class _AliasLoader(importlib.abc.Loader):
    def __init__(self, mod):
        self.mod = mod

    def create_module(self, spec):
        return self.mod

    def exec_module(self, module):
        pass


def install(workdir):
    """Install the finder; chdir into ``workdir`` (the reference opens logs/*.log relative to cwd)."""
    os.makedirs(os.path.join(workdir, "logs"), exist_ok=True)
    os.chdir(workdir)
    if not any(isinstance(f, _RefFinder) for f in sys.meta_path):
        sys.meta_path.insert(0, _RefFinder())
    logging.raiseExceptions = False
    import importlib
    mods = {}
    for name in ["log", "utils", "tree", "tu", "cu", "ctu", "sao", "image", "slice", "intra",
                 "scaling", "transform", "reconstruction", "pps", "sps", "cabac"]:
        mods[name] = importlib.import_module(name)
    mods["dec"] = importlib.import_module("dec")
    return mods


def silence(mods):
    lg = mods["log"]
    for n in ("main", "syntax", "cabac", "location", "qp", "intra"):
        getattr(lg, n).disabled = True

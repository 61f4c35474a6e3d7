"""Static check of the driver-facing scripts (bench.py, __graft_entry__.py): every name a function reads must be bound
somewhere it can be found -- its own scope, an enclosing function, the module, or builtins.  bench.py only runs on a
GPU box, so an undefined name there would otherwise surface only in the driver's run."""
import builtins
import os
import symtable

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _unbound(path):
    src = open(path).read()
    top = symtable.symtable(src, path, "exec")
    module_names = {s.get_name() for s in top.get_symbols() if s.is_assigned() or s.is_imported()}
    module_names |= {c.get_name() for c in top.get_children()} | {"__file__", "__name__", "__doc__"}
    bad = []

    def walk(t, enclosing):
        bound_here = {s.get_name() for s in t.get_symbols()
                      if s.is_assigned() or s.is_imported() or s.is_parameter()} if t.get_type() == "function" else set()
        for s in t.get_symbols():
            name = s.get_name()
            if t.get_type() != "function" or not s.is_referenced():
                continue
            if name in bound_here or s.is_free() and name in enclosing:
                continue
            if s.is_global() and (name in module_names or hasattr(builtins, name)):
                continue
            if s.is_free():
                continue
            bad.append("%s: %s" % (t.get_name(), name))
        for c in t.get_children():
            walk(c, enclosing | bound_here | ({c.get_name()} if t.get_type() == "function" else set()))

    for c in top.get_children():
        walk(c, set())
    return bad


@pytest.mark.parametrize("script", ["bench.py", "__graft_entry__.py"])
def test_no_unbound_names(script):
    assert _unbound(os.path.join(ROOT, script)) == []

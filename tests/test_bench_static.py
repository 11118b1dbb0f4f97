"""Static checks of bench.py's multi-rank report path (it only runs on GPU boxes with N > 1): the
rank's makeGraph shard [b, e) lives in one list, shard_be, bound once in main() and updated in place
by the per-step cost balancing, since the report divides by its length in shard mode (a loop variable
named e once crashed a 2-rank run).  No other name b or e is bound in main()."""
import ast
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bound_names(fn):
    out = []
    for node in ast.walk(fn):
        targets = []
        if isinstance(node, ast.Assign):
            targets = node.targets
        elif isinstance(node, (ast.AugAssign, ast.AnnAssign, ast.For, ast.comprehension)):
            targets = [node.target]
        elif isinstance(node, ast.withitem) and node.optional_vars is not None:
            targets = [node.optional_vars]
        elif isinstance(node, ast.ExceptHandler) and node.name:
            out.append(node.name)
        for t in targets:
            out.extend(_target_names(t))
    return out


def _target_names(t):
    """Names a target rebinds (x, (x, y), *x) -- not the containers of subscript / attribute stores."""
    if isinstance(t, ast.Name):
        return [t.id]
    if isinstance(t, (ast.Tuple, ast.List)):
        return [n for e in t.elts for n in _target_names(e)]
    if isinstance(t, ast.Starred):
        return _target_names(t.value)
    return []


def test_shard_range_names_bound_once_in_main():
    tree = ast.parse(open(os.path.join(REPO, "bench.py")).read())
    main = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "main")
    names = _bound_names(main)
    assert names.count("shard_be") == 1, names
    assert "b" not in names and "e" not in names, names

"""Static checks of bench.py's multi-rank report path (it only runs on GPU boxes with N > 1): the
rank's makeGraph shard (b, e) = shard_range(...) is bound once in main() and never rebound, since
the report divides by e - b in shard mode (a loop variable named e once crashed a 2-rank run)."""
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
            for n in ast.walk(t):
                if isinstance(n, ast.Name):
                    out.append(n.id)
    return out


def test_shard_range_names_bound_once_in_main():
    tree = ast.parse(open(os.path.join(REPO, "bench.py")).read())
    main = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "main")
    names = _bound_names(main)
    assert names.count("b") == 1 and names.count("e") == 1, names

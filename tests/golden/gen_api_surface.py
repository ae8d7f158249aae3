"""Generate tests/golden/api_surface.json: the parameter lists (names, kinds, default expressions) of the
reference's Python surface on the combine path, read from /root/reference as text with `ast` (nothing of
the reference is imported or executed).  tests/test_api_surface.py compares this build's signatures with it.

  python tests/golden/gen_api_surface.py      (in the build container, where /root/reference exists)
"""
import ast
import json
import os

REF = '/root/reference/deep_ep'
SOURCES = {'ElasticBuffer': 'buffers/elastic.py', 'EPHandle': 'buffers/elastic.py', 'EventOverlap': 'utils/event.py'}
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'api_surface.json')


def _params(f: ast.FunctionDef):
    a = f.args
    pos = a.posonlyargs + a.args
    defaults = [None] * (len(pos) - len(a.defaults)) + [ast.unparse(d) for d in a.defaults]
    out = [dict(name=p.arg, kind='positional', default=d) for p, d in zip(pos, defaults)]
    if a.vararg:
        out.append(dict(name=a.vararg.arg, kind='var_positional', default=None))
    for p, d in zip(a.kwonlyargs, a.kw_defaults):
        out.append(dict(name=p.arg, kind='keyword_only', default=None if d is None else ast.unparse(d)))
    if a.kwarg:
        out.append(dict(name=a.kwarg.arg, kind='var_keyword', default=None))
    return out


def main():
    surface = {}
    for cls, rel in SOURCES.items():
        path = os.path.join(REF, rel)
        tree = ast.parse(open(path).read())
        node = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == cls)
        methods = {}
        for f in node.body:
            if isinstance(f, ast.FunctionDef) and (not f.name.startswith('_') or f.name == '__init__'):
                methods[f.name] = dict(params=_params(f), line=f.lineno,
                                       decorators=[ast.unparse(d) for d in f.decorator_list])
        surface[cls] = dict(source=f'deep_ep/{rel}', methods=methods)
    json.dump(surface, open(OUT, 'w'), indent=1, sort_keys=True)
    print(f'wrote {OUT}: ' + ', '.join(f'{c} {len(v["methods"])} methods' for c, v in surface.items()))


if __name__ == '__main__':
    main()

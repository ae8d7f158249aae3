"""The drop-in boundary, checked mechanically: every method of the reference's Python surface on the
combine path (ElasticBuffer, EPHandle, EventOverlap; tests/golden/api_surface.json, generated from
/root/reference's sources by tests/golden/gen_api_surface.py) exists here with the same parameters in the
same order, of the same kind and with the same defaults.  Methods of the subsystems this build leaves out
(Engram, PP, AGRS: SURVEY.md section 8) are listed with that reason and must NOT be
half-present.  Additions beyond the reference are keyword-only parameters after its own.  CPU only."""
import inspect
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SURFACE = json.load(open(os.path.join(ROOT, 'tests', 'golden', 'api_surface.json')))

OUT_OF_SCOPE = {
    'ElasticBuffer': {'get_engram_storage_size_hint', 'engram_write', 'engram_fetch',            # Engram
                      'get_pp_buffer_size_hint', 'pp_set_config', 'pp_send', 'pp_recv',           # PP send / recv
                      'get_agrs_num_max_session_bytes', 'get_agrs_buffer_size_hint',              # AGRS all-gather
                      'create_agrs_session', 'destroy_agrs_session', 'agrs_new_session',
                      'agrs_set_config', 'agrs_get_inplace_tensor', 'all_gather'},
}


def _classes():
    import deep_ep
    return {'ElasticBuffer': deep_ep.ElasticBuffer, 'EPHandle': deep_ep.EPHandle, 'EventOverlap': deep_ep.EventOverlap}


_KIND = {inspect.Parameter.POSITIONAL_ONLY: 'positional', inspect.Parameter.POSITIONAL_OR_KEYWORD: 'positional',
         inspect.Parameter.VAR_POSITIONAL: 'var_positional', inspect.Parameter.KEYWORD_ONLY: 'keyword_only',
         inspect.Parameter.VAR_KEYWORD: 'var_keyword'}


def _ours(fn):
    fn = inspect.unwrap(fn)
    params = []
    for p in inspect.signature(fn).parameters.values():
        d = None if p.default is inspect.Parameter.empty else repr(p.default)
        params.append(dict(name=p.name, kind=_KIND[p.kind], default=d))
    return params


def _same_default(ref: str, ours: str) -> bool:
    if ref == ours:
        return True
    import ast
    try:
        return ast.literal_eval(ref) == ast.literal_eval(ours)
    except (ValueError, SyntaxError):
        return False


CASES = [(cls, name) for cls, v in SURFACE.items() for name in sorted(v['methods'])
         if name not in OUT_OF_SCOPE.get(cls, ())]


@pytest.mark.parametrize('cls,name', CASES)
def test_method_matches_the_reference(cls, name):
    ref = SURFACE[cls]['methods'][name]['params']
    ours_cls = _classes()[cls]
    assert hasattr(ours_cls, name), f'{cls}.{name} missing (reference {SURFACE[cls]["source"]}:' \
                                    f'{SURFACE[cls]["methods"][name]["line"]})'
    ours = _ours(getattr(ours_cls, name))
    if ref and ref[0]['name'] == 'self' and (not ours or ours[0]['name'] != 'self'):
        ref = ref[1:]                                   # a method the reference binds, here a staticmethod view
    assert [p['name'] for p in ours[:len(ref)]] == [p['name'] for p in ref], (cls, name, ours, ref)
    for r, o in zip(ref, ours):
        assert r['kind'] == o['kind'], (cls, name, r, o)
        assert (r['default'] is None) == (o['default'] is None), (cls, name, r, o)
        if r['default'] is not None:
            assert _same_default(r['default'], o['default']), (cls, name, r, o)
    for extra in ours[len(ref):]:                       # additions: keyword-only, with a default
        assert extra['kind'] == 'keyword_only' and extra['default'] is not None, (cls, name, extra)


def test_out_of_scope_methods_are_absent():
    classes = _classes()
    for cls, names in OUT_OF_SCOPE.items():
        for name in names:
            assert name in SURFACE[cls]['methods'], f'fixture lost {cls}.{name}'
            assert not hasattr(classes[cls], name), f'{cls}.{name} is out of scope but present'

"""Host GML front end: lexer, parser, evaluator, RenderArgs
dumps. Runs GML programs once per frame on the host and hands RenderArgs to
the renderer through the `render` hook, exactly like the reference's
EvalState.Render (internal/gml/evaluator.go:48)."""
from .evaluator import EvalState, GMLError, SurfaceFn, eval_surface_fn  # noqa: F401
from .printer import render_args_lines  # noqa: F401
from .syntax import ParseError  # noqa: F401


def _hook(out):
    def render(e, args):
        # ConvertRenderArgsToScene clones the state for the render threads
        # (raytracer.go:738-751); closure surfaces evaluate on that clone.
        args.state = e.clone()
        out.append((args, e))
    return render


def run_file(path, extensions=False):
    """Evaluate a .gml file; returns the list of (RenderArgs, EvalState) it
    rendered (in order) and the final EvalState. extensions=True enables the
    ICFP operators the reference lacks (cone, light, spotlight, real)."""
    out = []
    st = EvalState(render=_hook(out), extensions=extensions)
    st.parse_and_eval_file(path)
    return out, st


def run_text(text, extensions=False):
    out = []
    st = EvalState(render=_hook(out), extensions=extensions)
    st.parse_and_eval(text)
    return out, st

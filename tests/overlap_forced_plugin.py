"""Opt-in pytest plugin (`PYTHONPATH=tests pytest -p overlap_forced_plugin -m gpu`): every wcpt context, group ranks'
included, is created with WCPT_OPTION_FRAME_OVERLAP = 2, so the whole GPU suite renders through the frame-overlap pipes
wherever the megakernel's tiles are cost-ordered (and the wavefront's pipelines run on), whatever the frame size. The
suite's oracle and one-device comparisons then check the overlap's ordering everywhere (tests that set the option
themselves still do). Not loaded by default."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "wc-path-tracer_amd"))

import wcpt  # noqa: E402
from wcpt import renderer as _renderer  # noqa: E402

_init = _renderer.Context.__init__


def _forced_init(self, *args, **kwargs):
    _init(self, *args, **kwargs)
    self.set_option(wcpt._lib.OPTION_FRAME_OVERLAP, 2)


_renderer.Context.__init__ = _forced_init

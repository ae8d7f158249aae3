"""Stream events and the overlap wrapper.

EventHandle mirrors the reference's C++ EventHandle (csrc/utils/event.hpp:10-42):
a device event recorded on a stream, plus optional tensors kept alive until the
event has been waited on (EP_AVOID_RECORD_STREAM mode).  EventOverlap mirrors
deep_ep/utils/event.py:8-96 (same methods, same hook and context-manager behaviour).
"""
from typing import Any, Callable, Optional, Sequence

import torch


class EventHandle:
    """A device event recorded on `stream` (default: the current stream)."""

    def __init__(self, stream: Optional[torch.cuda.Stream] = None):
        stream = stream if stream is not None else torch.cuda.current_stream()
        self.event = torch.cuda.Event()
        self.event.record(stream)
        self.tensors_to_record: Optional[Sequence[Optional[torch.Tensor]]] = None

    def current_stream_wait(self) -> None:
        torch.cuda.current_stream().wait_event(self.event)

    def stream_wait(self, stream: torch.cuda.Stream) -> None:
        stream.wait_event(self.event)


class EventOverlap:
    """Wrapper of an EventHandle for overlapping communication with compute."""

    def __init__(self, event: Optional[EventHandle] = None,
                 extra_tensors: Optional[Sequence[torch.Tensor]] = None) -> None:
        self.event = event
        self.extra_tensors = extra_tensors
        self._release_handle_by_call = False
        self.hook_after_wait: Optional[Callable] = None

    def current_stream_wait(self, release_handle: bool = False) -> None:
        assert self.event is not None
        self.event.current_stream_wait()
        if self.hook_after_wait is not None:
            self.hook_after_wait()
            self.hook_after_wait = None
        if release_handle:
            self.event = None

    def register_hook_after_wait(self, hook_after_wait: Callable) -> None:
        assert self.hook_after_wait is None, 'A hook is already registered on this `EventOverlap`'
        self.hook_after_wait = hook_after_wait

    def __call__(self, release_handle: bool = False) -> 'EventOverlap':
        self._release_handle_by_call = release_handle
        return self

    def __enter__(self) -> Any:
        return self

    def __exit__(self, exc_type: Any, exc_val: Any, exc_tb: Any) -> None:
        if self.event is not None:
            self.current_stream_wait(release_handle=self._release_handle_by_call)
        self._release_handle_by_call = False

"""CPU restatement of the HTTP/1.x request-head step Envoy's codec performs
before the cilium.l7policy filter (cilium_l7policy.cc:127-170).  TEST
INFRASTRUCTURE ONLY.  Envoy's http_parser is external and not vendored, so
this follows RFC 7230 request-line / header-field grammar as that parser
enforces it; parity for this step is unpinned.  Written with
regular expressions, independently of csrc/http_parse.cc."""
from __future__ import annotations

import re

_TOKEN = rb"[!#$%&'*+\-.^_`|~0-9A-Za-z]+"
_REQ_LINE = re.compile(rb"(" + _TOKEN + rb") ([\x21-\x7e\x80-\xff]+) HTTP/[0-9]\.[0-9]\Z")
_FIELD = re.compile(rb"(" + _TOKEN + rb"):[ \t]*(.*?)[ \t]*\Z", re.S)
_BAD_VALUE = re.compile(rb"[\x00-\x08\x0a-\x1f\x7f]")


MAX_HEAD = 60 * 1024  # Envoy's default max_request_headers_kb


def parse_head(raw: bytes):
    """→ list of (name, value) as the filter sees them, or None if rejected."""
    if len(raw) > MAX_HEAD:
        return None
    end = raw.find(b"\r\n\r\n")
    if end < 0:
        # no empty line: an incomplete head
        return None
    lines = raw[:end].split(b"\r\n")
    m = _REQ_LINE.match(lines[0])
    if not m:
        return None
    out = [(b":method", m.group(1)), (b":path", m.group(2))]
    host, rest = None, []
    for ln in lines[1:]:
        f = _FIELD.match(ln)
        if not f or _BAD_VALUE.search(f.group(2)):
            return None
        name, value = f.group(1), f.group(2)
        if name.lower() == b"host":
            if host is None:
                host = value
        else:
            rest.append((name, value))
    if host is not None:
        out.append((b":authority", host))
    return out + rest

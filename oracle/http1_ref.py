"""CPU restatement of what stands between a raw HTTP/1.x request head and the
cilium.l7policy filter (envoy/cilium_l7policy.cc:127-170): Envoy's HTTP/1
codec (nodejs http_parser) and the connection manager's request checks.
TEST INFRASTRUCTURE ONLY.  Written with regular expressions over lines,
independently of csrc/http_parse.cc and the device parser.

Neither http_parser nor Envoy's source is vendored in the reference (Envoy is
pinned by SHA in envoy/WORKSPACE:10).  What is restated, and from where:

  http_parser (v2.8.x as Envoy pinned it in 2018, built with its default
  HTTP_PARSER_STRICT=1; restated from its state machine):
    s_start_req           CR / LF bytes before the request line are skipped
    s_req_method          the method is one of http_parser's method table
                          (METHODS below), matched case-sensitively
    s_req_spaces_before_url  one or more SP before the target
    parse_url_char        strict normal_url_char: target bytes 0x21-0x7E
                          ('?' and '#' are state changes that accept; bytes
                          >= 0x80, HTAB and FF are rejected when strict)
    s_req_http_*          "HTTP/" major "." minor, then CR LF or a bare LF
    s_req_line_almost_done / s_header_almost_done / s_headers_almost_done
                          a CR must be followed by LF; a bare LF ends a line
                          wherever CR LF does (request line, header lines,
                          the empty line that ends the head)
    s_header_field        a name is a run of tokens[] bytes (RFC 7230 tchar),
                          then ':' with nothing between
    s_header_value*       leading SP / HTAB discarded; value bytes
                          IS_HEADER_CHAR (HTAB, 0x20-0x7E, 0x80-0xFF)
    h_content_length      a non-empty Content-Length value is digits, then
                          SP only; a second non-empty one is an error; the
                          value may not pass (ULLONG_MAX - 10) / 10 before a
                          digit is appended
  Envoy (restated):
    codec_impl.cc onHeadersCompleteBase: a version other than 1.1 is
                          "HTTP/1.0" to the layers above; conn_manager_impl
                          answers it 426 unless accept_http_10 is set.  Cilium
                          sets no http_protocol_options (pkg/envoy/server.go:
                          172-215), and the option is off by default — the
                          vendored API says so (pkg/envoy/envoy/api/v2/core/
                          protocol.pb.go:108-112): only HTTP/1.1 heads reach
                          the filter
    conn_manager_impl.cc decodeHeaders: no Host → 400; a :path not starting
                          with '/' → 404 (absolute-form, authority-form and
                          asterisk-form targets all stop here)
    HTTP/1 codec          "host" is the :authority header; trailing OWS of a
                          value is not part of it; the first Host value is the
                          one the filter sees; max_request_headers_kb (60)
                          bounds the head

Still unpinned (no reference text or vector covers them; documented in
DESIGN.md §4): obs-fold continuation lines (http_parser joins them into the
previous value; here the head is rejected, so the request is denied), a
repeated Host (first value here), multi-digit versions that equal 1.1
("HTTP/1.01": rejected here), more than one SP before "HTTP/", and the 60 KiB
bound taken over the raw head rather than Envoy's header-map byte size."""
from __future__ import annotations

import re

# http_parser.h HTTP_METHOD_MAP (v2.8): the methods s_req_method accepts
METHODS = frozenset(m.encode() for m in (
    "DELETE", "GET", "HEAD", "POST", "PUT", "CONNECT", "OPTIONS", "TRACE",
    "COPY", "LOCK", "MKCOL", "MOVE", "PROPFIND", "PROPPATCH", "SEARCH", "UNLOCK",
    "BIND", "REBIND", "UNBIND", "ACL",
    "REPORT", "MKACTIVITY", "CHECKOUT", "MERGE",
    "M-SEARCH", "NOTIFY", "SUBSCRIBE", "UNSUBSCRIBE",
    "PATCH", "PURGE", "MKCALENDAR",
    "LINK", "UNLINK"))

_TOKEN = rb"[!#$%&'*+\-.^_`|~0-9A-Za-z]+"
_REQ_LINE = re.compile(rb"([A-Z-]+) +(/[\x21-\x7e]*) HTTP/1\.1\Z")
_FIELD = re.compile(rb"(" + _TOKEN + rb"):[ \t]*(.*?)[ \t]*\Z", re.S)
_BAD_VALUE = re.compile(rb"[\x00-\x08\x0a-\x1f\x7f]")
_CL_VALUE = re.compile(rb"([0-9]+) *\Z")
_CL_LIMIT = ((1 << 64) - 1 - 10) // 10

MAX_HEAD = 60 * 1024  # Envoy's default max_request_headers_kb


def _lines(raw: bytes):
    """The head's lines before its empty line (each ended by LF, one CR
    before the LF dropped), or None when the head is incomplete or a CR
    stands anywhere else."""
    body = raw.lstrip(b"\r\n")
    m = re.search(rb"\n\r?\n", body)
    if m is None:
        return None
    lines = []
    for ln in body[:m.start() + 1].split(b"\n")[:-1]:
        if ln.endswith(b"\r"):
            ln = ln[:-1]
        if b"\r" in ln:
            return None
        lines.append(ln)
    return lines


def _content_length_ok(raw_value: bytes, seen: bool):
    """h_content_length on the value after its leading SP / HTAB: → (ok,
    seen after it)."""
    if not raw_value:
        return True, seen  # an empty value never enters the CL states
    m = _CL_VALUE.match(raw_value)
    if m is None or seen:
        return False, True
    cl = 0
    for d in m.group(1):
        if cl > _CL_LIMIT:
            return False, True
        cl = cl * 10 + d - 48
    return True, True


def parse_head(raw: bytes):
    """→ list of (name, value) as the filter sees them, or None when the
    codec or the connection manager stops the request before the filter."""
    if len(raw) > MAX_HEAD:
        return None
    lines = _lines(raw)
    if not lines:
        return None
    m = _REQ_LINE.match(lines[0])
    if not m or m.group(1) not in METHODS:
        return None
    out = [(b":method", m.group(1)), (b":path", m.group(2))]
    host, rest, cl_seen = None, [], False
    for ln in lines[1:]:
        f = _FIELD.match(ln)
        if not f or _BAD_VALUE.search(f.group(2)):
            return None
        name, value = f.group(1), f.group(2)
        lname = name.lower()
        if lname == b"content-length":
            ok, cl_seen = _content_length_ok(ln[len(name) + 1:].lstrip(b" \t"), cl_seen)
            if not ok:
                return None
        if lname == b"host":
            if host is None:
                host = value
        else:
            rest.append((name, value))
    if host is None:
        return None  # conn_manager_impl: Host required
    out.append((b":authority", host))
    return out + rest

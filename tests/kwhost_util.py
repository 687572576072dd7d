"""Start / talk to the kwhost HTTP front (policy-server_amd/kwhost) in tests."""
import http.client
import json
import os
import socket
import subprocess
import tempfile
import time

from helpers import ROOT, config

KWHOST = os.path.join(ROOT, "policy-server_amd", "kwhost")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Host:
    """kwhost on 127.0.0.1 with configs/<name>.yml read by its native YAML reader (as_json: the
    same document as JSON; policies_file: any policies file); a context manager."""

    def __init__(self, name, extra=(), continue_on_errors=True, namespace="kubewarden", as_json=False,
                 policies_file=None):
        self.port = free_port()
        self.path = None
        if policies_file:
            path = policies_file
        elif as_json:
            fd, self.path = tempfile.mkstemp(suffix=".json")
            with os.fdopen(fd, "w") as f:
                json.dump(config(name), f)
            path = self.path
        else:
            path = os.path.join(ROOT, "configs", f"{name}.yml")
        args = [KWHOST, "--policies", path, "--port", str(self.port)]
        if continue_on_errors:
            args.append("--continue-on-errors")
        if namespace:
            args += ["--always-accept-admission-reviews-on-namespace", namespace]
        self.log = tempfile.TemporaryFile()
        self.proc = subprocess.Popen(args + list(extra), stdout=subprocess.DEVNULL, stderr=self.log)

    def __enter__(self):
        deadline = time.time() + 60
        while time.time() < deadline:
            if self.proc.poll() is not None:
                raise RuntimeError("kwhost exited: " + self.stderr())
            try:
                if self.request("GET", "/readiness")[0] == 200:
                    return self
            except OSError:
                time.sleep(0.05)
        raise RuntimeError("kwhost did not become ready")

    def stderr(self):
        self.log.seek(0)
        return self.log.read().decode(errors="replace")

    def __exit__(self, *a):
        rc = self.proc.poll()
        if rc is not None:  # died under the test: show why
            print(f"kwhost exit status {rc}; stderr:\n{self.stderr()}")
        self.proc.kill()  # the exact child this object started
        self.proc.wait(timeout=10)
        if self.path:
            os.unlink(self.path)

    def conn(self):
        return http.client.HTTPConnection("127.0.0.1", self.port, timeout=60)

    def request(self, method, path, body=None, ctype="application/json", conn=None, chunked=False):
        c = conn or self.conn()
        headers = {"Content-Type": ctype} if ctype else {}
        if chunked:
            headers["Transfer-Encoding"] = "chunked"
            data = body.encode() if isinstance(body, str) else body
            body = iter([data[i:i + 65536] for i in range(0, len(data), 65536)])
        c.request(method, path, body=body, headers=headers, encode_chunked=chunked)
        r = c.getresponse()
        data = r.read()
        if conn is None:
            c.close()
        return r.status, r.getheader("content-type"), data

"""SQLite-backed ML-Metadata-compatible store (types, artifacts, executions, events, contexts,
attributions, associations).

Reference contract: the MLMD read API used by `notebooks/utils.py:214-503` and
`notebooks/tfx_utils.py:50-65` (``get_events_by_artifact_ids``, ``get_artifacts_by_type``, ...),
plus the write path the TFX publisher performs for every component run (SURVEY §2.3 T10,
MLMD sqlite at ``<tfx_root>/metadata/<pipeline>/metadata.db``).
"""
from __future__ import annotations

import json
import os
import sqlite3
import threading
import time
from typing import Iterable, Sequence

from .proto import (Artifact, ArtifactState, ArtifactType, ConnectionConfig, Context, ContextType, Event,
                    EventPathStep, Execution, ExecutionState, ExecutionType, Value, _props)

_SCHEMA = """
CREATE TABLE IF NOT EXISTS Type (
  id INTEGER PRIMARY KEY AUTOINCREMENT, name TEXT NOT NULL, type_kind INTEGER NOT NULL,
  properties TEXT NOT NULL DEFAULT '{}', UNIQUE(name, type_kind));
CREATE TABLE IF NOT EXISTS Artifact (
  id INTEGER PRIMARY KEY AUTOINCREMENT, type_id INTEGER NOT NULL, uri TEXT, name TEXT, state INTEGER,
  properties TEXT NOT NULL DEFAULT '{}', custom_properties TEXT NOT NULL DEFAULT '{}',
  create_time INTEGER, update_time INTEGER);
CREATE INDEX IF NOT EXISTS idx_artifact_type ON Artifact(type_id);
CREATE INDEX IF NOT EXISTS idx_artifact_uri ON Artifact(uri);
CREATE TABLE IF NOT EXISTS Execution (
  id INTEGER PRIMARY KEY AUTOINCREMENT, type_id INTEGER NOT NULL, name TEXT, last_known_state INTEGER,
  properties TEXT NOT NULL DEFAULT '{}', custom_properties TEXT NOT NULL DEFAULT '{}',
  create_time INTEGER, update_time INTEGER);
CREATE INDEX IF NOT EXISTS idx_execution_type ON Execution(type_id);
CREATE TABLE IF NOT EXISTS Context (
  id INTEGER PRIMARY KEY AUTOINCREMENT, type_id INTEGER NOT NULL, name TEXT NOT NULL,
  properties TEXT NOT NULL DEFAULT '{}', custom_properties TEXT NOT NULL DEFAULT '{}',
  UNIQUE(type_id, name));
CREATE TABLE IF NOT EXISTS Event (
  id INTEGER PRIMARY KEY AUTOINCREMENT, artifact_id INTEGER NOT NULL, execution_id INTEGER NOT NULL,
  type INTEGER NOT NULL, path TEXT NOT NULL DEFAULT '[]', ms_since_epoch INTEGER);
CREATE INDEX IF NOT EXISTS idx_event_artifact ON Event(artifact_id);
CREATE INDEX IF NOT EXISTS idx_event_execution ON Event(execution_id);
CREATE TABLE IF NOT EXISTS Attribution (context_id INTEGER, artifact_id INTEGER, UNIQUE(context_id, artifact_id));
CREATE TABLE IF NOT EXISTS Association (context_id INTEGER, execution_id INTEGER, UNIQUE(context_id, execution_id));
"""

_EXECUTION, _ARTIFACT, _CONTEXT = 0, 1, 2


def _enc_props(p) -> str:
    out = {}
    for k, v in (p or {}).items():
        v = Value.of(v)
        kind = v.WhichOneof()
        if kind is None:
            continue
        out[k] = {"int_value": "i", "double_value": "d", "string_value": "s"}[kind] + ":" + json.dumps(v.value)
    return json.dumps(out, sort_keys=True)


def _dec_props(s: str):
    p = _props()
    for k, enc in json.loads(s or "{}").items():
        kind, raw = enc.split(":", 1)
        val = json.loads(raw)
        dict.__setitem__(p, k, Value(int_value=val) if kind == "i" else
                         Value(double_value=val) if kind == "d" else Value(string_value=val))
    return p


def _now_ms() -> int:
    return int(time.time() * 1000)


class MetadataStore:
    """MLMD-compatible metadata store on SQLite (thread-safe; one connection per store)."""

    def __init__(self, config: ConnectionConfig | str | None = None):
        if isinstance(config, str):
            path = config
        elif config is None or config.fake_database or not config.sqlite.filename_uri:
            path = ":memory:"
        else:
            path = config.sqlite.filename_uri
        if path != ":memory:":
            d = os.path.dirname(os.path.abspath(path))
            os.makedirs(d, exist_ok=True)
        self.path = path
        self._lock = threading.RLock()
        self._db = sqlite3.connect(path, check_same_thread=False, timeout=60)
        self._db.execute("PRAGMA journal_mode=WAL" if path != ":memory:" else "PRAGMA journal_mode=MEMORY")
        self._db.executescript(_SCHEMA)
        self._db.commit()

    def close(self):
        with self._lock:
            self._db.close()

    # ------------------------------------------------------------------ types
    def _put_type(self, t, kind: int, can_add_fields: bool = True) -> int:
        with self._lock:
            row = self._db.execute("SELECT id, properties FROM Type WHERE name=? AND type_kind=?",
                                   (t.name, kind)).fetchone()
            props = {k: int(v) for k, v in (t.properties or {}).items()}
            if row:
                old = json.loads(row[1])
                for k, v in props.items():
                    if k in old and old[k] != v:
                        raise ValueError(f"type {t.name}: property {k} changes type {old[k]} -> {v}")
                if not can_add_fields and set(props) - set(old):
                    raise ValueError(f"type {t.name}: new properties {set(props) - set(old)}")
                old.update(props)
                self._db.execute("UPDATE Type SET properties=? WHERE id=?", (json.dumps(old), row[0]))
                self._db.commit()
                return row[0]
            cur = self._db.execute("INSERT INTO Type(name, type_kind, properties) VALUES (?,?,?)",
                                   (t.name, kind, json.dumps(props)))
            self._db.commit()
            return cur.lastrowid

    def put_artifact_type(self, t: ArtifactType, can_add_fields: bool = True) -> int:
        t.id = self._put_type(t, _ARTIFACT, can_add_fields)
        return t.id

    def put_execution_type(self, t: ExecutionType, can_add_fields: bool = True) -> int:
        t.id = self._put_type(t, _EXECUTION, can_add_fields)
        return t.id

    def put_context_type(self, t: ContextType, can_add_fields: bool = True) -> int:
        t.id = self._put_type(t, _CONTEXT, can_add_fields)
        return t.id

    def _types(self, kind: int, where: str = "", args: Sequence = ()):
        cls = {_ARTIFACT: ArtifactType, _EXECUTION: ExecutionType, _CONTEXT: ContextType}[kind]
        with self._lock:
            rows = self._db.execute(f"SELECT id, name, properties FROM Type WHERE type_kind=? {where} ORDER BY id",
                                    (kind, *args)).fetchall()
        return [cls(name=n, properties=json.loads(p), id=i) for i, n, p in rows]

    def get_artifact_type(self, name: str) -> ArtifactType:
        r = self._types(_ARTIFACT, "AND name=?", (name,))
        if not r:
            raise KeyError(f"artifact type {name} not found")
        return r[0]

    def get_execution_type(self, name: str) -> ExecutionType:
        r = self._types(_EXECUTION, "AND name=?", (name,))
        if not r:
            raise KeyError(f"execution type {name} not found")
        return r[0]

    def get_context_type(self, name: str) -> ContextType:
        r = self._types(_CONTEXT, "AND name=?", (name,))
        if not r:
            raise KeyError(f"context type {name} not found")
        return r[0]

    def get_artifact_types(self):
        return self._types(_ARTIFACT)

    def get_execution_types(self):
        return self._types(_EXECUTION)

    def get_context_types(self):
        return self._types(_CONTEXT)

    def _types_by_id(self, kind, ids):
        ids = list(ids)
        if not ids:
            return []
        q = ",".join("?" * len(ids))
        return self._types(kind, f"AND id IN ({q})", ids)

    def get_artifact_types_by_id(self, ids: Iterable[int]):
        return self._types_by_id(_ARTIFACT, ids)

    def get_execution_types_by_id(self, ids: Iterable[int]):
        return self._types_by_id(_EXECUTION, ids)

    def get_context_types_by_id(self, ids: Iterable[int]):
        return self._types_by_id(_CONTEXT, ids)

    # ------------------------------------------------------------------ artifacts
    def put_artifacts(self, artifacts: Sequence[Artifact]) -> list[int]:
        ids = []
        now = _now_ms()
        with self._lock:
            for a in artifacts:
                if a.type_id is None:
                    raise ValueError("artifact.type_id is required")
                if a.id is None:
                    cur = self._db.execute(
                        "INSERT INTO Artifact(type_id, uri, name, state, properties, custom_properties, create_time,"
                        " update_time) VALUES (?,?,?,?,?,?,?,?)",
                        (a.type_id, a.uri, a.name, int(a.state), _enc_props(a.properties),
                         _enc_props(a.custom_properties), now, now))
                    a.id = cur.lastrowid
                    a.create_time_since_epoch = now
                else:
                    self._db.execute(
                        "UPDATE Artifact SET uri=?, name=?, state=?, properties=?, custom_properties=?, update_time=?"
                        " WHERE id=?", (a.uri, a.name, int(a.state), _enc_props(a.properties),
                                        _enc_props(a.custom_properties), now, a.id))
                a.last_update_time_since_epoch = now
                ids.append(a.id)
            self._db.commit()
        return ids

    @staticmethod
    def _row_to_artifact(r) -> Artifact:
        return Artifact(id=r[0], type_id=r[1], uri=r[2] or "", name=r[3], state=ArtifactState(r[4] or 0),
                        properties=_dec_props(r[5]), custom_properties=_dec_props(r[6]),
                        create_time_since_epoch=r[7] or 0, last_update_time_since_epoch=r[8] or 0)

    def _artifacts(self, where="", args=()):
        with self._lock:
            rows = self._db.execute(
                "SELECT id, type_id, uri, name, state, properties, custom_properties, create_time, update_time"
                f" FROM Artifact {where} ORDER BY id", args).fetchall()
        return [self._row_to_artifact(r) for r in rows]

    def get_artifacts(self):
        return self._artifacts()

    def get_artifacts_by_id(self, ids: Iterable[int]):
        ids = list(ids)
        if not ids:
            return []
        return self._artifacts(f"WHERE id IN ({','.join('?' * len(ids))})", ids)

    def get_artifacts_by_type(self, type_name: str):
        try:
            t = self.get_artifact_type(type_name)
        except KeyError:
            return []
        return self._artifacts("WHERE type_id=?", (t.id,))

    def get_artifacts_by_uri(self, uri: str):
        return self._artifacts("WHERE uri=?", (uri,))

    # ------------------------------------------------------------------ executions
    def put_executions(self, executions: Sequence[Execution]) -> list[int]:
        ids = []
        now = _now_ms()
        with self._lock:
            for e in executions:
                if e.type_id is None:
                    raise ValueError("execution.type_id is required")
                if e.id is None:
                    cur = self._db.execute(
                        "INSERT INTO Execution(type_id, name, last_known_state, properties, custom_properties,"
                        " create_time, update_time) VALUES (?,?,?,?,?,?,?)",
                        (e.type_id, e.name, int(e.last_known_state), _enc_props(e.properties),
                         _enc_props(e.custom_properties), now, now))
                    e.id = cur.lastrowid
                    e.create_time_since_epoch = now
                else:
                    self._db.execute(
                        "UPDATE Execution SET name=?, last_known_state=?, properties=?, custom_properties=?,"
                        " update_time=? WHERE id=?", (e.name, int(e.last_known_state), _enc_props(e.properties),
                                                      _enc_props(e.custom_properties), now, e.id))
                e.last_update_time_since_epoch = now
                ids.append(e.id)
            self._db.commit()
        return ids

    def _executions(self, where="", args=()):
        with self._lock:
            rows = self._db.execute(
                "SELECT id, type_id, name, last_known_state, properties, custom_properties, create_time, update_time"
                f" FROM Execution {where} ORDER BY id", args).fetchall()
        return [Execution(id=r[0], type_id=r[1], name=r[2], last_known_state=ExecutionState(r[3] or 0),
                          properties=_dec_props(r[4]), custom_properties=_dec_props(r[5]),
                          create_time_since_epoch=r[6] or 0, last_update_time_since_epoch=r[7] or 0) for r in rows]

    def get_executions(self):
        return self._executions()

    def get_executions_by_id(self, ids: Iterable[int]):
        ids = list(ids)
        if not ids:
            return []
        return self._executions(f"WHERE id IN ({','.join('?' * len(ids))})", ids)

    def get_executions_by_type(self, type_name: str):
        try:
            t = self.get_execution_type(type_name)
        except KeyError:
            return []
        return self._executions("WHERE type_id=?", (t.id,))

    # ------------------------------------------------------------------ events
    def put_events(self, events: Sequence[Event]) -> None:
        with self._lock:
            for ev in events:
                path = [{"index": s.index, "key": s.key} for s in ev.path]
                self._db.execute("INSERT INTO Event(artifact_id, execution_id, type, path, ms_since_epoch)"
                                 " VALUES (?,?,?,?,?)", (ev.artifact_id, ev.execution_id, int(ev.type),
                                                         json.dumps(path), ev.milliseconds_since_epoch or _now_ms()))
            self._db.commit()

    def _events(self, col, ids):
        ids = list(ids)
        if not ids:
            return []
        with self._lock:
            rows = self._db.execute(
                f"SELECT artifact_id, execution_id, type, path, ms_since_epoch FROM Event WHERE {col} IN "
                f"({','.join('?' * len(ids))}) ORDER BY id", ids).fetchall()
        return [Event(artifact_id=a, execution_id=e, type=Event.Type(t),
                      path=[EventPathStep(**s) for s in json.loads(p)], milliseconds_since_epoch=ms)
                for a, e, t, p, ms in rows]

    def get_events_by_artifact_ids(self, ids: Iterable[int]):
        return self._events("artifact_id", ids)

    def get_events_by_execution_ids(self, ids: Iterable[int]):
        return self._events("execution_id", ids)

    # ------------------------------------------------------------------ contexts
    def put_contexts(self, contexts: Sequence[Context]) -> list[int]:
        ids = []
        with self._lock:
            for c in contexts:
                if c.id is None:
                    row = self._db.execute("SELECT id FROM Context WHERE type_id=? AND name=?",
                                           (c.type_id, c.name)).fetchone()
                    if row:
                        c.id = row[0]
                if c.id is None:
                    cur = self._db.execute("INSERT INTO Context(type_id, name, properties, custom_properties)"
                                           " VALUES (?,?,?,?)", (c.type_id, c.name, _enc_props(c.properties),
                                                                 _enc_props(c.custom_properties)))
                    c.id = cur.lastrowid
                else:
                    self._db.execute("UPDATE Context SET properties=?, custom_properties=? WHERE id=?",
                                     (_enc_props(c.properties), _enc_props(c.custom_properties), c.id))
                ids.append(c.id)
            self._db.commit()
        return ids

    def _contexts(self, where="", args=()):
        with self._lock:
            rows = self._db.execute(f"SELECT id, type_id, name, properties, custom_properties FROM Context {where}"
                                    " ORDER BY id", args).fetchall()
        return [Context(id=r[0], type_id=r[1], name=r[2], properties=_dec_props(r[3]),
                        custom_properties=_dec_props(r[4])) for r in rows]

    def get_contexts(self):
        return self._contexts()

    def get_contexts_by_type(self, type_name: str):
        try:
            t = self.get_context_type(type_name)
        except KeyError:
            return []
        return self._contexts("WHERE type_id=?", (t.id,))

    def get_context_by_type_and_name(self, type_name: str, name: str) -> Context | None:
        r = [c for c in self.get_contexts_by_type(type_name) if c.name == name]
        return r[0] if r else None

    def put_attributions_and_associations(self, attributions: Sequence[tuple[int, int]],
                                          associations: Sequence[tuple[int, int]]) -> None:
        with self._lock:
            for ctx, art in attributions:
                self._db.execute("INSERT OR IGNORE INTO Attribution VALUES (?,?)", (ctx, art))
            for ctx, ex in associations:
                self._db.execute("INSERT OR IGNORE INTO Association VALUES (?,?)", (ctx, ex))
            self._db.commit()

    def get_artifacts_by_context(self, context_id: int):
        return self._artifacts("WHERE id IN (SELECT artifact_id FROM Attribution WHERE context_id=?)", (context_id,))

    def get_executions_by_context(self, context_id: int):
        return self._executions("WHERE id IN (SELECT execution_id FROM Association WHERE context_id=?)",
                                (context_id,))

    def get_contexts_by_artifact(self, artifact_id: int):
        return self._contexts("WHERE id IN (SELECT context_id FROM Attribution WHERE artifact_id=?)", (artifact_id,))

    def get_contexts_by_execution(self, execution_id: int):
        return self._contexts("WHERE id IN (SELECT context_id FROM Association WHERE execution_id=?)",
                              (execution_id,))

    # ------------------------------------------------------------------ composite
    def put_execution(self, execution: Execution, artifact_and_events: Sequence[tuple[Artifact, Event | None]],
                      contexts: Sequence[Context] = ()) -> tuple[int, list[int], list[int]]:
        """Atomically publish an execution with its input/output artifacts and events."""
        with self._lock:
            [eid] = self.put_executions([execution])
            arts = [a for a, _ in artifact_and_events]
            aids = self.put_artifacts(arts)
            evs = []
            for (a, ev), aid in zip(artifact_and_events, aids):
                if ev is not None:
                    ev.artifact_id, ev.execution_id = aid, eid
                    evs.append(ev)
            self.put_events(evs)
            cids = self.put_contexts(list(contexts)) if contexts else []
            self.put_attributions_and_associations([(c, a) for c in cids for a in aids], [(c, eid) for c in cids])
        return eid, aids, cids

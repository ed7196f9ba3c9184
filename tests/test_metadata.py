"""MLMD-compatible store: types, artifacts, executions, events, contexts, lineage search."""
import pytest

from mifx.metadata.lineage import ReadonlyMetadataStore
from mifx.metadata.proto import (Artifact, ArtifactType, ConnectionConfig, Context, ContextType, Event, EventPathStep,
                                 Execution, ExecutionType, INT, STRING)
from mifx.metadata.store import MetadataStore


def _store(tmp_path):
    cfg = ConnectionConfig()
    cfg.sqlite.filename_uri = str(tmp_path / "m.db")
    return MetadataStore(cfg)


def test_types_roundtrip_and_property_type_conflict(tmp_path):
    s = _store(tmp_path)
    t = ArtifactType(name="Data", properties={"split": STRING})
    tid = s.put_artifact_type(t)
    assert s.put_artifact_type(ArtifactType(name="Data", properties={"split": STRING, "n": INT})) == tid
    assert s.get_artifact_type("Data").properties == {"split": STRING, "n": INT}
    with pytest.raises(ValueError):
        s.put_artifact_type(ArtifactType(name="Data", properties={"split": INT}))
    with pytest.raises(KeyError):
        s.get_execution_type("nope")


def test_artifacts_executions_events_and_lineage(tmp_path):
    s = _store(tmp_path)
    at = s.put_artifact_type(ArtifactType(name="Examples", properties={"split": STRING}))
    mt_ = s.put_artifact_type(ArtifactType(name="Model"))
    et = s.put_execution_type(ExecutionType(name="trainer"))
    ex_a = Artifact(type_id=at, uri="/d/train")
    ex_a.properties["split"] = "train"
    [aid] = s.put_artifacts([ex_a])
    m = Artifact(type_id=mt_, uri="/m/1")
    m.custom_properties["acc"] = 0.9
    e = Execution(type_id=et)
    ctype = s.put_context_type(ContextType(name="run"))
    eid, aids, cids = s.put_execution(e, [(ex_a, Event(type=Event.INPUT, path=[EventPathStep(key="examples")])),
                                          (m, Event(type=Event.OUTPUT))], [Context(type_id=ctype, name="r1")])
    assert aids[0] == aid
    got = s.get_artifacts_by_id([m.id])[0]
    assert got.custom_properties["acc"].double_value == pytest.approx(0.9)
    assert got.properties["missing"].WhichOneof() is None
    evs = s.get_events_by_execution_ids([eid])
    assert {ev.type for ev in evs} == {Event.INPUT, Event.OUTPUT}
    assert evs[0].path[0].key == "examples"
    assert [a.uri for a in s.get_artifacts_by_type("Examples")] == ["/d/train"]
    assert s.get_executions_by_type("trainer")[0].id == eid
    assert len(s.get_artifacts_by_context(cids[0])) == 2
    ro = ReadonlyMetadataStore(s)
    assert ro.get_source_artifact_of_type(m.id, "Examples").uri == "/d/train"
    assert ro.get_dest_artifact_of_type(aid, "Model").uri == "/m/1"
    assert ro.get_execution_for_output_artifact(m.id, "trainer").id == eid
    df = ro.get_artifact_df(m.id)
    assert df.loc[m.id, "Type"] == "Model"
    g = ro.get_artifact_lineage(m.id)
    assert set(g.nodes) == {m.id, -eid, aid}


def test_in_memory_store():
    s = MetadataStore()
    t = s.put_execution_type(ExecutionType(name="x"))
    [i] = s.put_executions([Execution(type_id=t)])
    assert s.get_executions_by_id([i])[0].id == i

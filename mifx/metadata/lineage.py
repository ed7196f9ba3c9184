"""Read-only lineage/analysis helpers over the metadata store.

Parity with `notebooks/utils.py:51-503` (ReadonlyMetadataStore, _LineageGraphHelper) and
`notebooks/tfx_utils.py:28-203` (TFXReadonlyMetadataStore): DataFrame views of artifacts and
executions, recursive source/destination artifact search through events, execution lookup for
an output artifact, property comparisons, and a bipartite lineage graph (artifact node ids
positive, execution node ids negative) with optional matplotlib plotting.
"""
from __future__ import annotations

import json
import os

import pandas as pd

from .proto import ConnectionConfig, Event, is_input_event, is_output_event
from .store import MetadataStore


def _value_str(v) -> str:
    k = v.WhichOneof()
    return "" if k is None else str(getattr(v, k))


class LineageGraphHelper:
    def __init__(self, store: MetadataStore):
        self.store = store

    def upstream_execution_ids(self, artifact_id: int) -> list[int]:
        return [e.execution_id for e in self.store.get_events_by_artifact_ids([artifact_id]) if is_output_event(e)]

    def upstream_artifact_ids(self, execution_id: int) -> list[int]:
        return [e.artifact_id for e in self.store.get_events_by_execution_ids([execution_id]) if is_input_event(e)]

    def get_artifact_lineage(self, artifact_id: int, max_depth: int | None = None):
        import networkx as nx

        g = nx.DiGraph()
        self._add_node(g, artifact_id, 0, True)
        self._add_parents(g, artifact_id, True, 1, max_depth)
        return g

    def _add_node(self, g, node_id: int, depth: int, is_artifact: bool):
        if is_artifact:
            a = self.store.get_artifacts_by_id([node_id])[0]
            t = self.store.get_artifact_types_by_id([a.type_id])[0]
            label = f"{t.name}\n{a.id}"
            g.add_node(node_id, depth=depth, is_artifact=True, label=label, uri=a.uri)
        else:
            e = self.store.get_executions_by_id([-node_id])[0]
            t = self.store.get_execution_types_by_id([e.type_id])[0]
            g.add_node(node_id, depth=depth, is_artifact=False, label=f"{t.name}\n{e.id}")

    def _add_parents(self, g, node_id, is_artifact, depth, max_depth):
        if max_depth is not None and depth > max_depth:
            return
        if is_artifact:
            for eid in self.upstream_execution_ids(node_id):
                if -eid not in g:
                    self._add_node(g, -eid, depth, False)
                g.add_edge(-eid, node_id)
                self._add_parents(g, -eid, False, depth + 1, max_depth)
        else:
            for aid in self.upstream_artifact_ids(-node_id):
                if aid not in g:
                    self._add_node(g, aid, depth, True)
                g.add_edge(aid, node_id)
                self._add_parents(g, aid, True, depth + 1, max_depth)

    def plot_artifact_lineage(self, g, path: str | None = None):
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        import networkx as nx

        depth = nx.get_node_attributes(g, "depth")
        maxd = max(depth.values()) if depth else 0
        pos = {}
        layers: dict[int, list] = {}
        for n, d in depth.items():
            layers.setdefault(d, []).append(n)
        for d, nodes in layers.items():
            for i, n in enumerate(sorted(nodes)):
                pos[n] = (maxd - d, i - len(nodes) / 2)
        colors = ["c" if g.nodes[n]["is_artifact"] else "m" for n in g.nodes]
        fig = plt.figure(figsize=(max(6, 2.5 * (maxd + 1)), 5))
        nx.draw(g, pos, labels=nx.get_node_attributes(g, "label"), node_color=colors, node_size=2200,
                font_size=7, arrows=True)
        if path:
            fig.savefig(path)
        return fig


class ReadonlyMetadataStore:
    def __init__(self, store: MetadataStore):
        self.store = store
        self._lineage = LineageGraphHelper(store)

    # ------------------------------------------------------------------ dataframes
    def get_df_from_single_artifact_or_execution(self, obj) -> dict:
        d = {"ID": obj.id, "Type": self._type_name(obj)}
        if hasattr(obj, "uri"):
            d["URI"] = obj.uri
        for k, v in obj.properties.items():
            d[k] = _value_str(v)
        for k, v in obj.custom_properties.items():
            d[k] = _value_str(v)
        return d

    def _type_name(self, obj) -> str:
        if hasattr(obj, "uri"):
            return self.store.get_artifact_types_by_id([obj.type_id])[0].name
        return self.store.get_execution_types_by_id([obj.type_id])[0].name

    def get_df_from_artifacts_or_executions(self, objects) -> pd.DataFrame:
        df = pd.DataFrame([self.get_df_from_single_artifact_or_execution(o) for o in objects])
        if len(df):
            df = df.set_index("ID")
        df.index.name = "ID"
        return df

    def get_artifact_df(self, artifact_id: int) -> pd.DataFrame:
        return self.get_df_from_artifacts_or_executions(self.store.get_artifacts_by_id([artifact_id]))

    def get_execution_df(self, execution_id: int) -> pd.DataFrame:
        return self.get_df_from_artifacts_or_executions(self.store.get_executions_by_id([execution_id]))

    def get_artifacts_of_type_df(self, type_name: str) -> pd.DataFrame:
        return self.get_df_from_artifacts_or_executions(self.store.get_artifacts_by_type(type_name))

    def get_executions_of_type_df(self, type_name: str) -> pd.DataFrame:
        return self.get_df_from_artifacts_or_executions(self.store.get_executions_by_type(type_name))

    # ------------------------------------------------------------------ lineage search
    def get_source_artifact_of_type(self, artifact_id: int, source_type_name: str):
        """Walk input events upstream (BFS) until an artifact of `source_type_name` is found."""
        try:
            want = self.store.get_artifact_type(source_type_name).id
        except KeyError:
            return None
        seen, frontier = {artifact_id}, [artifact_id]
        while frontier:
            nxt = []
            for aid in frontier:
                for eid in self._lineage.upstream_execution_ids(aid):
                    for src in self._lineage.upstream_artifact_ids(eid):
                        if src in seen:
                            continue
                        seen.add(src)
                        a = self.store.get_artifacts_by_id([src])[0]
                        if a.type_id == want:
                            return a
                        nxt.append(src)
            frontier = nxt
        return None

    def get_dest_artifact_of_type(self, artifact_id: int, dest_type_name: str):
        """Walk output events downstream (BFS) until an artifact of `dest_type_name` is found."""
        try:
            want = self.store.get_artifact_type(dest_type_name).id
        except KeyError:
            return None
        seen, frontier = {artifact_id}, [artifact_id]
        while frontier:
            nxt = []
            for aid in frontier:
                for ev in self.store.get_events_by_artifact_ids([aid]):
                    if not is_input_event(ev):
                        continue
                    for out in self.store.get_events_by_execution_ids([ev.execution_id]):
                        if not is_output_event(out) or out.artifact_id in seen:
                            continue
                        seen.add(out.artifact_id)
                        a = self.store.get_artifacts_by_id([out.artifact_id])[0]
                        if a.type_id == want:
                            return a
                        nxt.append(out.artifact_id)
            frontier = nxt
        return None

    def get_execution_for_output_artifact(self, artifact_id: int, type_name: str):
        for ev in self.store.get_events_by_artifact_ids([artifact_id]):
            if is_output_event(ev):
                ex = self.store.get_executions_by_id([ev.execution_id])[0]
                if self.store.get_execution_types_by_id([ex.type_id])[0].name == type_name:
                    return ex
        return None

    def display_artifact_and_execution_properties(self, artifact_id: int, execution_type_name: str) -> pd.DataFrame:
        a = self.get_artifact_df(artifact_id)
        ex = self.get_execution_for_output_artifact(artifact_id, execution_type_name)
        if ex is None:
            return a
        e = self.get_df_from_artifacts_or_executions([ex])
        return pd.concat([a.T, e.T], axis=0, keys=["artifact", "execution"])

    def compare_artifact_pair_and_execution_properties(self, artifact_id: int, other_artifact_id: int,
                                                       execution_type_name: str) -> pd.DataFrame:
        left = self.display_artifact_and_execution_properties(artifact_id, execution_type_name)
        right = self.display_artifact_and_execution_properties(other_artifact_id, execution_type_name)
        return pd.concat([left, right], axis=1)

    def get_artifact_lineage(self, artifact_id: int, max_depth: int | None = None):
        return self._lineage.get_artifact_lineage(artifact_id, max_depth)

    def plot_artifact_lineage(self, artifact_id: int, max_depth: int | None = None, path: str | None = None):
        return self._lineage.plot_artifact_lineage(self.get_artifact_lineage(artifact_id, max_depth), path)


class TFXArtifactTypes:
    EXAMPLES = "ExamplesPath"
    SCHEMA = "SchemaPath"
    EXAMPLE_STATS = "ExampleStatisticsPath"
    EXAMPLE_VALIDATION = "ExampleValidationPath"
    TRANSFORMED_EXAMPLES = "TransformPath"
    MODEL = "ModelExportPath"
    MODEL_EVAL = "ModelEvalPath"
    MODEL_BLESSING = "ModelBlessingPath"
    PUSHED_MODEL = "ModelPushPath"


class TFXExecutionTypes:
    EXAMPLE_GEN = "examples_gen"
    STATISTICS_GEN = "statistics_gen"
    SCHEMA_GEN = "schema_gen"
    EXAMPLE_VALIDATION = "example_validation"
    TRANSFORM = "transform"
    TRAINER = "trainer"
    EVALUATOR = "evaluator"
    MODEL_VALIDATOR = "model_validator"
    PUSHER = "pusher"


class TFXReadonlyMetadataStore(ReadonlyMetadataStore):
    """TFX-typed wrapper (`notebooks/tfx_utils.py:50-203`)."""

    @staticmethod
    def from_sqlite_db(filename_uri: str) -> "TFXReadonlyMetadataStore":
        cfg = ConnectionConfig()
        cfg.sqlite.filename_uri = filename_uri
        return TFXReadonlyMetadataStore(MetadataStore(cfg))

    def _read_json(self, artifact_id: int, name: str):
        a = self.store.get_artifacts_by_id([artifact_id])[0]
        p = os.path.join(a.uri, name)
        with open(p) as f:
            return json.load(f)

    def get_tfma_analysis(self, model_id: int, slicing_column: str | None = None) -> pd.DataFrame:
        """Sliced metrics of the evaluation that consumed `model_id` (cf. display_tfma_analysis)."""
        ev = self.get_dest_artifact_of_type(model_id, TFXArtifactTypes.MODEL_EVAL)
        if ev is None:
            raise ValueError(f"no evaluation found for model {model_id}")
        from ..evaluator.metrics import load_eval_result

        return load_eval_result(ev.uri).slice_frame(slicing_column)

    display_tfma_analysis = get_tfma_analysis

    def compare_tfma_analysis(self, model_id: int, other_model_id: int) -> pd.DataFrame:
        a = self.get_tfma_analysis(model_id)
        b = self.get_tfma_analysis(other_model_id)
        return pd.concat([a, b], axis=1, keys=[f"model_{model_id}", f"model_{other_model_id}"])

    def get_stats_for_examples(self, examples_id: int) -> dict:
        st = self.get_dest_artifact_of_type(examples_id, TFXArtifactTypes.EXAMPLE_STATS)
        if st is None:
            raise ValueError(f"no statistics for examples {examples_id}")
        from ..components.statistics import load_statistics

        return load_statistics(st.uri)

    display_stats_for_examples = get_stats_for_examples

    def compare_stats_for_examples(self, examples_id: int, other_examples_id: int, split: str = "train"):
        from ..components.statistics import stats_frame

        a = stats_frame(self.get_stats_for_examples(examples_id), split)
        b = stats_frame(self.get_stats_for_examples(other_examples_id), split)
        return pd.concat([a, b], axis=1, keys=[f"examples_{examples_id}", f"examples_{other_examples_id}"])

    def get_examples_stats_for_model(self, model_id: int) -> dict:
        ex = self.get_source_artifact_of_type(model_id, TFXArtifactTypes.EXAMPLES)
        if ex is None:
            raise ValueError(f"no examples upstream of model {model_id}")
        return self.get_stats_for_examples(ex.id)

    display_examples_stats_for_model = get_examples_stats_for_model

    def compare_examples_stats_for_models(self, model_id: int, other_model_id: int):
        a = self.get_source_artifact_of_type(model_id, TFXArtifactTypes.EXAMPLES)
        b = self.get_source_artifact_of_type(other_model_id, TFXArtifactTypes.EXAMPLES)
        return self.compare_stats_for_examples(a.id, b.id)

    def tensorboard_logdirs(self, model_id: int, *other_model_ids: int) -> str:
        """Comma-joined `name:path` logdir spec for the models' training logs (display_tensorboard)."""
        parts = []
        for mid in (model_id,) + other_model_ids:
            a = self.store.get_artifacts_by_id([mid])[0]
            parts.append(f"model_{mid}:{os.path.join(a.uri, 'logs')}")
        return ",".join(parts)

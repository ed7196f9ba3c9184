"""Data validation (TFDV-equivalent): statistics, schema inference, anomalies, skew/drift.

Reference notebooks: `02_TensorFlow_Data_Validation.ipynb`, `06_Airflow_Feature_Analysis.ipynb`."""
from .schema import (Feature, FloatDomain, IntDomain, Schema, StringDomain, load_schema_text,  # noqa: F401
                     write_schema_text)
from .stats import (generate_statistics_from_csv, generate_statistics_from_dataframe,  # noqa: F401
                    generate_statistics_from_table, get_feature_stats, load_statistics, stats_frame,
                    visualize_statistics, write_stats)
from .validate import (Anomalies, display_anomalies, infer_schema, linf_distance, set_domain,  # noqa: F401
                       summarize_l_inf, validate_statistics)


def get_feature(schema: Schema, name: str) -> Feature:
    return schema.get_feature(name)


def get_domain(schema: Schema, name: str):
    return schema.get_domain(name)


def display_schema(schema: Schema) -> str:
    import pandas as pd

    rows = []
    for f in schema.feature:
        d = schema.get_domain(f)
        dom = f"'{f.domain}'" if f.domain else ("int" if f.int_domain else "-")
        pres = "required" if (f.presence_min_fraction or 0) >= 1 else "optional"
        rows.append({"Feature name": f.name, "Type": f.type, "Presence": pres,
                     "Valency": "single" if f.univalent_shape or f.value_count_max == 1 else "-", "Domain": dom})
        _ = d
    txt = pd.DataFrame(rows).to_string(index=False)
    doms = "\n".join(f"{d.name}: {', '.join(d.value)}" for d in schema.string_domain)
    return txt + ("\n\n" + doms if doms else "")

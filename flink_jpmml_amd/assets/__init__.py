"""Model fixtures: Iris k-means PMML documents in every dialect the reference's tests load.

The reference ships them as XML assets (`A/*.xml`, table in SURVEY §2.3). We *generate* equivalent
documents (same centres, fields, versions/namespaces and quirks) so tests and examples are
self-contained on any machine:

========================  =========================================================
name                      distinguishing feature
========================  =========================================================
kmeans                    PMML 4.3, 4 clusters, Output ``PCluster`` (entityId)
kmeans41 / kmeans40       PMML 4.1 (4 clusters) / 4.0 (3 clusters)
kmeans42                  PMML 4.2, 3 clusters without ``size``
kmeans32                  PMML 3.2 with a header ``Extension``, clusters named "1".."3"
kmeans_nooutput           no ``<Output>``
kmeans_nooutput_notarget  no ``<Output>`` and no predicted field → ``EmptyScore``
kmeans_stringfields       active fields categorical/string (+Interval) → preparation fails
kmeans_empty              no ``<PMML>`` element → loading fails
========================  =========================================================
"""

from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

IRIS_FIELDS = ["sepal_length", "sepal_width", "petal_length", "petal_width"]
IRIS_INTERVALS = [(4.3, 7.9), (2.0, 4.4), (1.0, 6.9), (0.1, 2.5)]
IRIS_CLASSES = ["Iris-setosa", "Iris-versicolor", "Iris-virginica"]

# k-means centres (KNIME, 4 clusters) — the model every reference golden is computed on
CENTERS_4 = [
    [6.9125000000000005, 3.099999999999999, 5.846874999999999, 2.1312499999999996],
    [6.23658536585366, 2.8585365853658535, 4.807317073170731, 1.6219512195121943],
    [5.005999999999999, 3.4180000000000006, 1.464, 0.2439999999999999],
    [5.529629629629629, 2.6222222222222222, 3.940740740740741, 1.2185185185185188],
]
SIZES_4 = [32, 41, 50, 27]
# k-means centres (3 clusters; Spark MLlib / Rattle exports)
CENTERS_3 = [
    [6.8538461538461535, 3.076923076923076, 5.715384615384614, 2.0538461538461537],
    [5.883606557377049, 2.740983606557377, 4.388524590163936, 1.4344262295081966],
    [5.005999999999999, 3.4180000000000006, 1.4640000000000002, 0.2439999999999999],
]


def _ns(version: str) -> str:
    return "http://www.dmg.org/PMML-" + version.replace(".", "_")


def kmeans_pmml(
    version: str = "4.3",
    centers: Sequence[Sequence[float]] = CENTERS_4,
    sizes: Optional[Sequence[int]] = SIZES_4,
    names: Optional[Sequence[str]] = None,
    with_output: bool = True,
    with_target: bool = True,
    string_fields: bool = False,
    intervals: bool = True,
    invalid_treatment: Optional[str] = "asIs",
    header_extension: bool = False,
    application: str = "flink_jpmml_amd",
) -> str:
    """Render an Iris ``ClusteringModel`` PMML document."""
    k = len(centers)
    names = list(names) if names is not None else [f"cluster_{i}" for i in range(k)]
    lines: List[str] = ['<?xml version="1.0" encoding="UTF-8"?>',
                        f'<PMML version="{version}" xmlns="{_ns(version)}">']
    lines.append(' <Header copyright="generated">')
    if header_extension:
        lines.append('  <Extension name="user" value="generated" extender="flink_jpmml_amd"/>')
    lines.append(f'  <Application name="{application}" version="0.1"/>')
    lines.append(' </Header>')
    lines.append(f' <DataDictionary numberOfFields="{len(IRIS_FIELDS) + 1}">')
    for f, (lo, hi) in zip(IRIS_FIELDS, IRIS_INTERVALS):
        optype, dtype = ("categorical", "string") if string_fields else ("continuous", "double")
        if intervals:
            lines.append(f'  <DataField name="{f}" optype="{optype}" dataType="{dtype}">')
            lines.append(f'   <Interval closure="closedClosed" leftMargin="{lo}" rightMargin="{hi}"/>')
            lines.append('  </DataField>')
        else:
            lines.append(f'  <DataField name="{f}" optype="{optype}" dataType="{dtype}"/>')
    lines.append('  <DataField name="clazz" optype="categorical" dataType="string">')
    for c in IRIS_CLASSES:
        lines.append(f'   <Value value="{c}"/>')
    lines.append('  </DataField>')
    lines.append(' </DataDictionary>')
    lines.append(f' <ClusteringModel modelName="k-means" functionName="clustering" modelClass="centerBased" '
                 f'numberOfClusters="{k}">')
    lines.append('  <MiningSchema>')
    ivt = f' invalidValueTreatment="{invalid_treatment}"' if invalid_treatment else ""
    for f in IRIS_FIELDS:
        lines.append(f'   <MiningField name="{f}"{ivt}/>')
    if with_target:
        lines.append('   <MiningField name="clazz" invalidValueTreatment="asIs" usageType="predicted"/>')
    lines.append('  </MiningSchema>')
    lines.append('  <ComparisonMeasure kind="distance"><squaredEuclidean/></ComparisonMeasure>')
    for f in IRIS_FIELDS:
        lines.append(f'  <ClusteringField field="{f}" compareFunction="absDiff"/>')
    for i, c in enumerate(centers):
        size = f' size="{sizes[i]}"' if sizes else ""
        arr = " ".join(repr(float(x)) for x in c)
        lines.append(f'  <Cluster name="{names[i]}"{size}><Array n="{len(c)}" type="real">{arr}</Array></Cluster>')
    if with_output:
        lines.append('  <Output>')
        lines.append('   <OutputField name="PCluster" optype="categorical" dataType="string" targetField="clazz" '
                     'feature="entityId"/>')
        lines.append('  </Output>')
    lines.append(' </ClusteringModel>')
    lines.append('</PMML>')
    return "\n".join(lines) + "\n"


FIXTURES = {
    "kmeans": lambda: kmeans_pmml("4.3"),
    "kmeans41": lambda: kmeans_pmml("4.1"),
    "kmeans40": lambda: kmeans_pmml("4.0", CENTERS_3, [24, 33, 48]),
    "kmeans42": lambda: kmeans_pmml("4.2", CENTERS_3, None, intervals=False, invalid_treatment=None),
    "kmeans32": lambda: kmeans_pmml("3.2", CENTERS_3, [24, 33, 48], names=["1", "2", "3"], intervals=False,
                                    invalid_treatment=None, header_extension=True),
    "kmeans_nooutput": lambda: kmeans_pmml("4.3", with_output=False),
    "kmeans_nooutput_notarget": lambda: kmeans_pmml("4.3", with_output=False, with_target=False),
    "kmeans_stringfields": lambda: kmeans_pmml("4.3", string_fields=True),
    "kmeans_empty": lambda: "<!-- an empty model file: no PMML element -->\n",
}


def write_fixtures(directory: str) -> Dict[str, str]:
    """Write every fixture as ``<directory>/<name>.xml``; returns ``name -> path``."""
    os.makedirs(directory, exist_ok=True)
    out = {}
    for name, gen in FIXTURES.items():
        path = os.path.join(directory, f"{name}.xml")
        with open(path, "w") as fh:
            fh.write(gen())
        out[name] = path
    return out

"""Deploy artefacts (reference: helm/templates/*.yaml, helm/values.yaml):
the k8s manifests parse, every ConfigMap key is a setting the service reads,
the API pod runs one front door with one replica per GPU it requests, probes
hit real routes, Prometheus scrapes the API and the Pushgateway the ingest
Job pushes to, and the bare-metal launcher serves one front door."""
from pathlib import Path

import yaml

from githubrepostorag_amd.config import Settings
from githubrepostorag_amd.service.api import create_app

ROOT = Path(__file__).resolve().parents[1] / "deploy"


def _docs(name):
    return [d for d in yaml.safe_load_all((ROOT / "k8s" / name).read_text()) if d]


def _settings_envs():
    import inspect

    src = inspect.getsource(Settings)
    import re

    return set(re.findall(r'_(?:env|int|float|bool)\("([A-Z_]+)"', src)) | set(re.findall(r'os\.environ\.get\("([A-Z_]+)"', src))


def test_configmap_keys_are_read_by_settings():
    cm = next(d for d in _docs("rag-mi355x.yaml") if d["kind"] == "ConfigMap")
    unknown = set(cm["data"]) - _settings_envs()
    assert not unknown, f"ConfigMap keys nothing reads: {unknown}"


def test_api_pod_runs_front_door_over_its_gpus():
    dep = next(d for d in _docs("rag-mi355x.yaml") if d["kind"] == "Deployment" and d["metadata"]["name"] == "rag-api")
    c = dep["spec"]["template"]["spec"]["containers"][0]
    cmd = c["command"]
    assert cmd[:4] == ["python", "-m", "githubrepostorag_amd", "serve"]
    n = int(cmd[cmd.index("--replicas") + 1])
    assert n == int(c["resources"]["limits"]["amd.com/gpu"])
    cm = next(d for d in _docs("rag-mi355x.yaml") if d["kind"] == "ConfigMap")
    assert int(cm["data"]["DP"]) == n
    routes = {r.path for r in create_app().routes}
    for probe in ("readinessProbe", "livenessProbe"):
        assert c[probe]["httpGet"]["path"] in routes
    assert dep["spec"]["template"]["metadata"]["annotations"]["prometheus.io/path"] in routes


def test_monitoring_scrapes_api_and_pushgateway():
    docs = _docs("monitoring.yaml")
    prom = yaml.safe_load(next(d for d in docs if d["kind"] == "ConfigMap")["data"]["prometheus.yml"])
    targets = {t for job in prom["scrape_configs"] for sc in job["static_configs"] for t in sc["targets"]}
    cm = next(d for d in _docs("rag-mi355x.yaml") if d["kind"] == "ConfigMap")
    assert cm["data"]["PUSHGATEWAY_ADDRESS"] in targets
    assert "rag-api:8000" in targets
    svcs = {d["metadata"]["name"] for d in docs if d["kind"] == "Service"}
    assert {"pushgateway", "prometheus"} <= svcs


def test_launcher_serves_one_front_door():
    sh = (ROOT / "launch_node.sh").read_text()
    serve = sh.split("serve)")[1].split(";;")[0]
    assert "--replicas" in serve and serve.count("githubrepostorag_amd serve") == 1


def test_ingest_job_runs_dp_ingest_into_the_shared_volume():
    """The ingest Job (reference helm/templates/ingest-job.yaml: one batch run writing the vector store the
    workers read) is data-parallel over the GPUs it requests and writes the shard snapshots to the volume
    the API pod's replicas load from: its command parses with the CLI's own parser, --dp equals its GPU
    limit and the API pod's replica count, and INDEX_DIR lies on the PVC both pods mount."""
    from githubrepostorag_amd.cli import build_parser

    docs = _docs("rag-mi355x.yaml")
    job = next(d for d in docs if d["kind"] == "Job")
    spec = job["spec"]["template"]["spec"]
    c = spec["containers"][0]
    cmd = c["command"]
    assert cmd[:3] == ["python", "-m", "githubrepostorag_amd"]
    args = build_parser().parse_args(cmd[3:])
    assert args.cmd == "ingest" and args.source == "github" and args.dev_force_standalone
    assert args.dp == int(c["resources"]["limits"]["amd.com/gpu"])
    api = next(d for d in docs if d["kind"] == "Deployment" and d["metadata"]["name"] == "rag-api")
    acmd = api["spec"]["template"]["spec"]["containers"][0]["command"]
    assert args.dp == int(acmd[acmd.index("--replicas") + 1])
    cm = next(d for d in docs if d["kind"] == "ConfigMap")["data"]
    assert cm.get("INDEX_SHARDING", "shard") == "shard"  # replicas load shard-r-of-N snapshots
    claim = {v["persistentVolumeClaim"]["claimName"] for v in spec["volumes"] if "persistentVolumeClaim" in v}
    aspec = api["spec"]["template"]["spec"]
    assert claim and claim <= {v["persistentVolumeClaim"]["claimName"] for v in aspec.get("volumes", [])
                               if "persistentVolumeClaim" in v}
    mounts = [m["mountPath"] for m in c["volumeMounts"]]
    assert any(cm["INDEX_DIR"].startswith(m) for m in mounts)


def test_launcher_ingest_is_data_parallel():
    sh = (ROOT / "launch_node.sh").read_text()
    ingest = sh.split("ingest)")[1].split(";;")[0]
    assert "--dp" in ingest and "HIP_VISIBLE_DEVICES=0" not in ingest

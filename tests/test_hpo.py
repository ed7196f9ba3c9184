"""HPO: StudyJob parsing (incl. the Katib go-template worker), suggestions, trial execution."""
import sys

from mifx.hpo import GridSuggestion, ParameterConfig, RandomSuggestion, StudyRunner, StudySpec, parse_metrics

_STUDY = {
    "apiVersion": "kubeflow.org/v1alpha1", "kind": "StudyJob", "metadata": {"name": "rs"},
    "spec": {"studyName": "rs", "optimizationtype": "maximize", "objectivevaluename": "Validation-accuracy",
             "optimizationgoal": 0.99, "requestcount": 4, "metricsnames": ["accuracy"],
             "parameterconfigs": [
                 {"name": "--lr", "parametertype": "double", "feasible": {"min": "0.01", "max": "0.03"}},
                 {"name": "--num-layers", "parametertype": "int", "feasible": {"min": "2", "max": "5"}},
                 {"name": "--optimizer", "parametertype": "categorical", "feasible": {"list": ["sgd", "adam", "ftrl"]}}],
             "suggestionSpec": {"suggestionAlgorithm": "random", "requestNumber": 3},
             "workerSpec": {"goTemplate": {"rawTemplate": (
                 "apiVersion: batch/v1\nkind: Job\nmetadata:\n  name: {{.WorkerID}}\nspec:\n  template:\n    spec:\n"
                 "      containers:\n      - name: {{.WorkerID}}\n        image: img\n        command:\n"
                 "        - \"python\"\n        - \"/train.py\"\n        - \"--batch-size=64\"\n"
                 "        {{- with .HyperParameters}}\n        {{- range .}}\n        - \"{{.Name}}={{.Value}}\"\n"
                 "        {{- end}}\n        {{- end}}\n      restartPolicy: Never\n")}}}}


def test_parse_study_and_go_template():
    s = StudySpec.from_dict(_STUDY)
    assert (s.request_count, s.request_number, s.objective, s.goal) == (4, 3, "Validation-accuracy", 0.99)
    assert s.command == ["python", "/train.py", "--batch-size=64"]
    assert [p.parametertype for p in s.parameters] == ["double", "int", "categorical"]


def test_suggestions_respect_feasible_space():
    s = StudySpec.from_dict(_STUDY)
    for p in RandomSuggestion(s.parameters, 1).get(200):
        assert 0.01 <= p["--lr"] <= 0.03 and 2 <= p["--num-layers"] <= 5 and p["--optimizer"] in ("sgd", "adam", "ftrl")
    grid = GridSuggestion([ParameterConfig("a", "int", 1, 3), ParameterConfig("b", "categorical", values=["x", "y"])])
    assert len(grid.get(100)) == 6


def test_parse_metrics_last_value_wins():
    log = "epoch 1 accuracy=0.5\nValidation-accuracy=0.61\nepoch 2 accuracy=0.7 Validation-accuracy=0.72\n"
    assert parse_metrics(log, ["accuracy", "Validation-accuracy"]) == {"accuracy": 0.7, "Validation-accuracy": 0.72}


def test_in_process_trials_and_early_stop(tmp_path):
    s = StudySpec.from_dict(_STUDY)
    seen = []

    def trial(params, device):
        seen.append(device)
        return {"Validation-accuracy": 0.995 if params["--optimizer"] == "adam" else 0.5}

    res = StudyRunner(s, trial, workdir=str(tmp_path), num_gpus=2).run()
    assert res["goal_reached"] and res["best"]["params"]["--optimizer"] == "adam"
    assert len(res["trials"]) % 3 == 0 and len(res["trials"]) <= 12
    assert set(seen) <= {"0", "1"}


def test_subprocess_trials(tmp_path):
    worker = tmp_path / "w.py"
    worker.write_text("import sys\nargs=dict(a.split('=') for a in sys.argv[1:] if '=' in a)\n"
                      "print('accuracy=%s' % (1 - abs(float(args['--lr']) - 0.02)))\n"
                      "print('Validation-accuracy=%s' % (1 - abs(float(args['--lr']) - 0.02)))\n")
    d = dict(_STUDY)
    d["spec"] = dict(_STUDY["spec"], requestcount=2, optimizationgoal=2.0, workerSpec={"command": [sys.executable,
                                                                                                    str(worker)]})
    res = StudyRunner(StudySpec.from_dict(d), workdir=str(tmp_path), num_gpus=0).run()
    assert len(res["trials"]) == 6 and all(t["status"] == "Succeeded" for t in res["trials"])
    assert res["best"]["metrics"]["Validation-accuracy"] == max(t["metrics"]["Validation-accuracy"]
                                                                for t in res["trials"])

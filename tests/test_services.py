"""Jobs service, DAG operators, Hive warehouse, Elasticsearch index, project/dataset (CPU).

Reference behaviour: jobs-client/spark/jobs_spark_client.py (create_job/start_job),
airflow/launch_jobs.py:130 (task0 >> [task1, task2] >> sensor >> task3),
notebooks/hive/PyHive.ipynb (external CSV table -> partitioned ORC table -> queries),
notebooks/spark/Elasticsearch-python.ipynb (write a DataFrame, read it back)."""
import shutil
import textwrap
from pathlib import Path

import pandas as pd
import pytest

SACRAMENTO = Path("/root/reference/notebooks/featurestore/aws/data/Sacramentorealestatetransactions.csv")


def _prog(project_root, name, body):
    p = project_root / "Resources" / name
    p.parent.mkdir(parents=True, exist_ok=True)
    p.write_text(textwrap.dedent(body))
    return f"hdfs:///Projects/demo/Resources/{name}"


def test_jobs_lifecycle(project_root):
    from hops_examples_amd import jobs

    app = _prog(project_root, "pi.py", """
        import sys
        n = int(sys.argv[1])
        print("pi ~", sum(4 * (-1) ** k / (2 * k + 1) for k in range(n)))
    """)
    jobs.create_job("pi", {"appPath": app, "jobType": "PYSPARK"})
    ex = jobs.start_job("pi", "1000")
    s = jobs.wait_for_execution("pi", ex["id"], timeout=60)
    assert s["state"] == "FINISHED" and s["finalStatus"] == "SUCCEEDED"
    assert "pi ~ 3.14" in jobs.get_logs("pi")
    bad = _prog(project_root, "bad.py", "raise SystemExit(3)\n")
    jobs.create_job("bad", {"appPath": bad})
    e2 = jobs.start_job("bad")
    s2 = jobs.wait_for_execution("bad", e2["id"], timeout=60)
    assert s2["finalStatus"] == "FAILED" and s2["exitCode"] == 3
    assert [j["name"] for j in jobs.get_jobs()] == ["bad", "pi"]


def test_flink_runner_lifecycle_and_rest_client(project_root):
    """hops.beam runner lifecycle and the Flink REST flow of jobs-client/flink/jobs_flink_client.py:
    the runner is a job that becomes RUNNING once its REST endpoint is up (polled like the reference's
    90 s loop), a second client reuses it, programs are uploaded and run in task slots, REST errors
    raise RestAPIError with the reference's message shape, stop ends the runner job."""
    from hops_examples_amd import beam, jobs
    from hops_examples_amd.exceptions import RestAPIError

    app = project_root / "Resources" / "wordcount.py"
    app.parent.mkdir(parents=True, exist_ok=True)
    app.write_text(textwrap.dedent("""
        import collections, sys, time
        words = sys.argv[1:] or "the quick brown fox jumps over the lazy dog the end".split()
        print(dict(collections.Counter(words).most_common(1)))
        time.sleep(float(__import__("os").environ.get("WC_SLEEP", "0")))
    """))
    beam.create_runner("flinkrunner", num_of_taskmanagers=1, num_task_slots=1)
    assert beam.find_running("flinkrunner") is None
    with pytest.raises(RuntimeError):
        beam.run_pipeline("flinkrunner", str(app))
    beam.start_runner("flinkrunner")
    e = beam.wait_until_running("flinkrunner", wait=60, step=0.1)
    assert e is not None and beam.get_runner_state("flinkrunner") == "RUNNING"
    assert beam.find_running("flinkrunner")["endpoint"] == e["endpoint"]  # reuse, no second cluster
    ov = beam.overview(e["endpoint"])
    assert ov["slots-total"] == 1 and ov["jobs-running"] == 0
    r = beam.run_pipeline("flinkrunner", str(app), args="a b b c")
    s = beam.wait_job(r["endpoint"], r["jobid"], timeout=60)
    assert s["state"] == "FINISHED" and s["exit-code"] == 0
    with pytest.raises(RestAPIError, match="HTTP code: 404"):
        beam.run_program(e["endpoint"], "no_such_program.py")
    beam.stop_runner("flinkrunner")
    ex = jobs.wait_for_execution("flinkrunner", jobs.get_executions("flinkrunner")[-1]["id"], timeout=30)
    assert ex["state"] == "KILLED" and beam.find_running("flinkrunner") is None


def test_dag_job_chain_and_failure_propagation(project_root):
    from hops_examples_amd import jobs
    from hops_examples_amd.orchestration import DAG, HopsworksJobSuccessSensor, HopsworksLaunchOperator

    out = project_root / "order.txt"
    for i in range(4):
        app = _prog(project_root, f"job{i}.py", f"""
            import time
            time.sleep(0.2 if {i} == 2 else 0)
            open({str(out)!r}, "a").write("job-{i}\\n")
        """)
        jobs.create_job(f"job-{i}", {"appPath": app})
    dag = DAG("job_launcher_dag", schedule_interval="@once")
    t0 = HopsworksLaunchOperator(dag=dag, task_id="run_job-0", job_name="job-0")
    t1 = HopsworksLaunchOperator(dag=dag, task_id="run_job-1", job_name="job-1", wait_for_completion=False)
    t2 = HopsworksLaunchOperator(dag=dag, task_id="run_job-2", job_name="job-2", wait_for_completion=False)
    t3 = HopsworksLaunchOperator(dag=dag, task_id="run_job-3", job_name="job-3")
    sensor = HopsworksJobSuccessSensor(dag=dag, task_id="wait_for_job-2", job_name="job-2", timeout=60)
    t0 >> [t1, t2] >> sensor >> t3
    st = dag.run()
    assert set(st.values()) == {"success"}
    lines = out.read_text().split()
    assert lines[0] == "job-0" and lines.index("job-2") < lines.index("job-3")

    bad = _prog(project_root, "fail.py", "raise SystemExit(1)\n")
    jobs.create_job("fails", {"appPath": bad})
    dag2 = DAG("d2")
    a = HopsworksLaunchOperator(dag=dag2, task_id="a", job_name="fails")
    b = HopsworksLaunchOperator(dag=dag2, task_id="b", job_name="job-0")
    a >> b
    assert dag2.run() == {"a": "failed", "b": "upstream_failed"}


@pytest.mark.skipif(not SACRAMENTO.exists(), reason="reference fixture missing")
def test_hive_external_to_partitioned_orc(project_root):
    from hops_examples_amd import hive

    raw = project_root / "RawData"
    raw.mkdir(parents=True)
    lines = SACRAMENTO.read_text().splitlines()[1:]  # the notebook's external table has no header row
    (raw / "sacramento.csv").write_text("\n".join(lines) + "\n")
    h = hive.setup_hive_connection()
    h.execute("""CREATE EXTERNAL TABLE sacramento_properties_ext(
        street string, city string, zip int, state string, beds int, baths int, sq__ft float,
        sales_type string, sale_date string, price float, latitude float, longitude float)
        ROW FORMAT DELIMITED FIELDS TERMINATED BY ',' LOCATION '/Projects/demo/RawData'""")
    assert len(h.execute("select * from sacramento_properties_ext limit 10")) == 10
    h.execute("""CREATE TABLE sacramento_properties(street string, city string, state string, beds int,
        baths int, sq__ft float, sales_type string, sale_date string, price float, latitude float,
        longitude float) PARTITIONED by (zip int) STORED AS ORC""")
    h.execute("set hive.exec.dynamic.partition=true; set hive.exec.dynamic.partition.mode=nonstrict;")
    h.execute("""INSERT OVERWRITE TABLE sacramento_properties PARTITION (zip)
        SELECT street, city, state, beds, baths, sq__ft, sales_type, sale_date, price, latitude, longitude, zip
        FROM sacramento_properties_ext""")
    assert set(h.execute("show tables").tab_name) == {"sacramento_properties", "sacramento_properties_ext"}
    df = pd.read_csv(SACRAMENTO).rename(columns={"type": "sales_type"})
    got = h.execute("select sales_type, avg(price) as avg_price FROM sacramento_properties WHERE zip=95608 "
                    "GROUP BY sales_type LIMIT 10")
    exp = df[df.zip == 95608].groupby("sales_type").price.mean()
    for r in got.itertuples():
        assert abs(r.avg_price - exp[r.sales_type]) < 1e-6
    import pyarrow.orc as orc

    part = project_root / "Hive" / "warehouse" / "default.db" / "sacramento_properties" / "zip=95608"
    t = orc.read_table(str(next(part.glob("*.orc"))))
    assert t.num_rows == int((df.zip == 95608).sum())
    # overwrite replaces only the partitions present in the new data
    h.execute("INSERT OVERWRITE TABLE sacramento_properties PARTITION (zip) SELECT street, city, state, beds, "
              "baths, sq__ft, sales_type, sale_date, price, latitude, longitude, zip FROM sacramento_properties_ext "
              "WHERE zip = 95608")
    assert h.execute("select count(*) as n from sacramento_properties").n[0] == len(df)
    condos = h.cursor().execute("select * from sacramento_properties where `sales_type` = 'Condo'").fetchall()
    assert len(condos) == int((df.sales_type == "Condo").sum())


def test_elasticsearch_index_roundtrip(project_root):
    from hops_examples_amd import elasticsearch as es

    cfg = es.get_elasticsearch_config("Newsgroup")
    assert cfg["es.resource"] == "newsgroup/_doc"
    df = pd.DataFrame({"id": [1, 2, 3], "text": ["GPU kernels are fast", "hello world", "fast cars"],
                       "score": [3, 5, 9]})
    assert es.write(df, "newsgroup", id_field="id") == 3
    assert list(es.read("newsgroup", {"query": {"match": {"text": "fast"}}}).id) == [1, 3]
    q = {"query": {"bool": {"must": [{"range": {"score": {"gte": 4}}}], "must_not": [{"term": {"id": 3}}]}}}
    assert list(es.read("newsgroup", q).id) == [2]
    es.write(pd.DataFrame({"id": [1], "text": ["updated"], "score": [0]}), "newsgroup", id_field="id")
    assert len(es.read("newsgroup")) == 3


def test_project_and_dataset_upload(project_root, tmp_path):
    from hops_examples_amd import dataset, hdfs, project

    info = project.connect("demo", "localhost", port=443, api_key="not-a-real-key")
    assert "not-a-real-key" not in str(info)
    f = tmp_path / "prog.py"
    f.write_text("print(1)\n")
    dst = dataset.upload(str(f), "Resources")
    assert hdfs.exists("Resources/prog.py") and Path(dst).read_text() == "print(1)\n"
    d2 = dataset.download("Resources/prog.py", str(tmp_path / "dl"))
    assert Path(d2).exists()
    shutil.rmtree(tmp_path / "dl")

# %% [markdown]
# # Flink-style job client: start (or reuse) a runner, upload a program, run it
# Mirrors jobs-client/flink/jobs_flink_client.py: look for a running cluster with the job's name;
# otherwise `beam.create_runner` + `beam.start_runner` and wait up to 90 s (5 s steps) until it is
# RUNNING; upload the program (`POST /jars/upload`), run it (`POST /jars/<id>/run?entry-class=…&
# program-args=…`), surface REST errors as `RestAPIError`; `stop` stops the cluster.  There is no
# JVM here: the "jar" is a Python program (a .py file, or a .zip + entry-class module).
# %%
import argparse
import os
import sys
import textwrap

from hops_examples_amd import beam, hdfs
from hops_examples_amd.exceptions import RestAPIError

ap = argparse.ArgumentParser()
ap.add_argument("-j", "--job", default="flinkcluster")
ap.add_argument("-jar", default=None, help="program to run (default: a generated word count)")
ap.add_argument("-m", "--main", default="", help="entry module of a .zip program")
ap.add_argument("-tm", "--task-managers", default="1")
ap.add_argument("-yjm", "--yarnjobManagerMemory", default="2048")
ap.add_argument("-ytm", "--yarntaskManagerMemory", default="4096")
ap.add_argument("-ys", "--yarnslots", default="1")
ap.add_argument("-args", "--job-arguments", default="the quick brown fox jumps over the lazy dog the end")
ap.add_argument("action", nargs=argparse.REMAINDER)
args = ap.parse_args([] if "ipykernel" in sys.modules else sys.argv[1:])

if "stop" in args.action:
    beam.stop_runner(args.job)
    print("Stopped Flink cluster.")
    sys.exit(0)

# %%
wait = float(os.environ.get("HOPSX_RUNNER_WAIT_S", "90"))
running = beam.find_running(args.job)
if running is None:
    beam.create_runner(args.job, args.yarnjobManagerMemory, args.task_managers, args.yarntaskManagerMemory,
                       args.yarnslots)
    print("Waiting for flink cluster to start...")
    beam.start_runner(args.job)
    running = beam.wait_until_running(args.job, wait=wait, step=min(5.0, wait / 18))
    if running is None:
        print("Flink cluster did not start, check job logs for details")
        sys.exit(1)
    print("app_id: " + running["appId"])
    print("Flink cluster started successfully. Will now proceed to submit the job.")
else:
    print("Found Flink cluster with this name already running, will use it to submit the Flink job")

# %%
jar = args.jar
if jar is None:
    jar = os.path.join(hdfs.project_path(), "Resources", "wordcount.py")
    os.makedirs(os.path.dirname(jar), exist_ok=True)
    with open(jar, "w") as f:
        f.write(textwrap.dedent("""
            import collections, sys
            print(dict(collections.Counter(sys.argv[1:]).most_common(1)))
        """))
ep = running["endpoint"]
prog = beam.upload_program(ep, jar)
print("Submitting job to: " + ep + "/jars/" + prog + "/run")
try:
    job = beam.run_program(ep, prog, args.main, args.job_arguments)
except RestAPIError as e:
    print(e)
    sys.exit(1)
print("Flink job was submitted successfully:", beam.wait_job(ep, job))
beam.stop_runner(args.job)

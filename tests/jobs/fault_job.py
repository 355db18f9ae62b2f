"""Worker / PS of the fault-injection test (tests/test_fault_cpu.py): Hogwild-style SGD on the
reference's toy problem with the variables on the PS, MonitoredTrainingSession checkpointing every
5 steps.  Run the PS with DTG_FAULT=kill_ps_at_step:N; the harness restarts it."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import dtg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--job_name", default="worker")
    ap.add_argument("--task_index", type=int, default=0)
    ap.add_argument("--cluster", required=True)
    ap.add_argument("--logdir", required=True)
    ap.add_argument("--last_step", type=int, default=60)
    ap.add_argument("--step_sleep", type=float, default=0.01)
    a, _ = ap.parse_known_args()
    cluster = dtg.ClusterSpec(json.loads(a.cluster))
    server = dtg.Server(cluster, job_name=a.job_name, task_index=a.task_index)
    if a.job_name == "ps":
        server.join()
        return
    with dtg.device(dtg.train.replica_device_setter(ps_tasks=1, worker_device="/job:worker/task:%d" % a.task_index)):
        x = dtg.Variable([-1.0, 2.0], name="Variable")
        y = dtg.Variable([3.0, 0.5], name="Variable_1")
        c = x + y
        target = dtg.constant([100.0, 100.0])
        loss = dtg.reduce_mean(dtg.square(c - target))
        gs = dtg.train.get_or_create_global_step()
        train_op = dtg.train.GradientDescentOptimizer(1e-3).minimize(loss, global_step=gs)
    hooks = [dtg.train.StopAtStepHook(last_step=a.last_step)]
    steps = 0
    with dtg.train.MonitoredTrainingSession(master=server.target, is_chief=True, checkpoint_dir=a.logdir,
                                            save_checkpoint_steps=5, hooks=hooks) as sess:
        while not sess.should_stop():
            _, g = sess.run([train_op, gs])
            steps += 1
            time.sleep(a.step_sleep)  # paced so the PS's fault trigger fires mid-run
    print("RESULT " + json.dumps({"final_step": int(g), "local_runs": steps,
                                  "restored_from": sess.restored_from}), flush=True)


if __name__ == "__main__":
    main()

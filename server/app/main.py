"""Control-plane FastAPI app (reference server/app/main.py:28-126).

Lifespan: create tables, start the task-guarantee sweeper (dead workers,
stale jobs), close the geo client on shutdown.  Routers: jobs, workers,
admin; ``/metrics`` + ``/ready`` from the observability service; the admin
dashboard page is served at ``/admin``.
"""
from __future__ import annotations

import asyncio
import logging
from contextlib import asynccontextmanager
from pathlib import Path

from fastapi import FastAPI
from fastapi.middleware.cors import CORSMiddleware
from fastapi.responses import FileResponse
from fastapi.staticfiles import StaticFiles

from app.api import admin, jobs, workers
from app.config import settings
from app.db.database import SessionLocal, init_db
from app.services import geo
from app.services.geo import REGION_NAMES
from app.services.observability import setup_metrics_routes
from app.services.task_guarantee import TaskGuaranteeBackgroundWorker

logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(name)s - %(levelname)s - %(message)s")
logger = logging.getLogger(__name__)

task_guarantee_worker = TaskGuaranteeBackgroundWorker(SessionLocal)

REGION_DESCRIPTIONS = {
    "asia-east": "China, Japan, Korea", "asia-south": "Singapore, Thailand, Vietnam, India",
    "europe-west": "Germany, France, UK", "europe-east": "Poland, Eastern Europe",
    "america-north": "USA, Canada", "america-south": "Brazil, Argentina", "oceania": "Australia, New Zealand",
}


@asynccontextmanager
async def lifespan(app: FastAPI):
    init_db()
    logger.info("starting control plane in region %s", settings.region)
    bg = asyncio.create_task(task_guarantee_worker.start())
    try:
        yield
    finally:
        task_guarantee_worker.stop()
        bg.cancel()
        try:
            await bg
        except (asyncio.CancelledError, Exception):
            pass
        await geo.cleanup_resources()
        logger.info("server shutdown complete")


app = FastAPI(title=settings.app_name, description="Distributed GPU inference control plane (MI355X workers)",
              version="1.0.0", lifespan=lifespan)
app.add_middleware(CORSMiddleware, allow_origins=["*"], allow_credentials=True, allow_methods=["*"],
                   allow_headers=["*"])
app.include_router(jobs.router)
app.include_router(workers.router)
app.include_router(admin.router)
setup_metrics_routes(app)

STATIC_DIR = Path(__file__).resolve().parent.parent / "static"
if STATIC_DIR.exists():
    app.mount("/static", StaticFiles(directory=str(STATIC_DIR)), name="static")


@app.get("/admin")
@app.get("/admin/{path:path}")
async def admin_spa(path: str = ""):
    index = STATIC_DIR / "admin" / "index.html"
    if index.exists():
        return FileResponse(index)
    return {"error": "Admin panel not found"}


@app.get("/")
async def root():
    return {"message": "Distributed GPU Inference API", "version": "1.0.0", "region": settings.region}


@app.get("/health")
async def health():
    return {"status": "healthy", "region": settings.region}


@app.get("/regions")
async def get_regions():
    return {"current_region": settings.region,
            "available_regions": [{"code": c, "name": REGION_NAMES[c], "description": REGION_DESCRIPTIONS[c]}
                                  for c in REGION_NAMES]}


if __name__ == "__main__":
    import uvicorn
    uvicorn.run(app, host="0.0.0.0", port=8000)
